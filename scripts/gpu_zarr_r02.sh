# Row f2 loop: Zarr GPU parity tests + the bench's Zarr line (+ kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-z}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_zarr.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && echo tests ok || { echo tests FAIL; tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o zarr --output-format csv -- python3 scripts/zarr_bench.py > gpurun_out/$T/zarr.json 2> gpurun_out/$T/zarr.err && echo zarr ok || { echo zarr FAIL; tail -30 gpurun_out/$T/zarr.err; exit 1; }
cat gpurun_out/$T/zarr.json
