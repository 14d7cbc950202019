# Phase profile (noise, fake) and the headline bench line alone (no secondary lines).
set -o pipefail
TAG=${1:-quick}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for g in noise fake; do
  timeout -k 10 200 python -u scripts/phase_profile.py $g 4096 > $O/phase_$g.log 2>&1 && tail -4 $O/phase_$g.log || { echo phase FAIL; tail -20 $O/phase_$g.log; exit 1; }
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/bench.json 2> $O/bench.err && cat $O/bench.json || { echo bench FAIL; tail -20 $O/bench.err; exit 1; }
