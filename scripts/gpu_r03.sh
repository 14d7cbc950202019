# One GPU call of round 3: parity tests, smoke, the full bench line, and the rocprofv3
# kernel-trace summary of the headline (same command, --no-extra).
# Usage (from the repo root on the box): bash scripts/gpu_r03.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_residency.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_residency.log 2>&1 && echo residency ok || { echo residency FAIL; tail -60 $O/pytest_residency.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo tests ok || { echo tests FAIL; tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok || { echo smoke FAIL; tail -20 $O/smoke.log; exit 1; }
fi
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err && echo bench ok || { echo bench FAIL; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
PBX_KSTREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/prof_bench.json 2> $O/prof.log && echo prof ok || { echo prof FAIL; tail -30 $O/prof.log; exit 1; }
find $O/prof -name "*stats*"
