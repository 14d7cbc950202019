# One GPU call: parity tests, smoke, bench line, rocprofv3 kernel-trace stats of the bench.
# Usage (from the repo root on the box): bash scripts/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
O=gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo tests ok || { echo tests FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok || { echo smoke FAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && echo bench ok || { echo bench FAIL; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/prof_bench.json 2> $O/prof.log && echo prof ok || { echo prof FAIL; tail -30 $O/prof.log; exit 1; }
find $O/prof -name "*stats*"
# row f2: kernel trace of the Zarr decode workload (k_zarr_*)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_zarr -o zarr --output-format csv -- python3 scripts/zarr_bench.py > $O/prof_zarr.json 2> $O/prof_zarr.log && echo zarr prof ok || { echo zarr prof FAIL; tail -30 $O/prof_zarr.log; exit 1; }
