# Headline bench line with 1 vs 3 kernel streams, alternating, ROUNDS rounds.
set -o pipefail
TAG=${1:-kstreams}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
for i in $(seq ${ROUNDS:-2}); do
  for k in 3 1 2; do
    PBX_KSTREAMS=$k timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/bench_k${k}_$i.json 2> $O/bench_k${k}_$i.err || exit 1
    python3 -c "import json,sys; b=json.load(open(sys.argv[1])); print(sys.argv[2], b['value'], b['ms_per_step'], b['kernel_streams']['serial_pass_tiles_per_s'])" $O/bench_k${k}_$i.json k$k | tee -a $O/summary.txt
  done
done
