# k_filter3 check: the PNG filter parity tests, then the filter kernels' timing (k_filter3 and,
# for comparison, k_filter2), then a kernel trace of k_filter3.
set -o pipefail
TAG=${1:-filt}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_zarr.py tests/test_tiff_tiled.py -x -v -m gpu --timeout 200 --timeout-method thread -k "filter or adaptive or sweep or checksum or tiled" > $O/pytest_filter.log 2>&1 && echo filter tests ok || { echo filter tests FAIL; tail -40 $O/pytest_filter.log; exit 1; }
timeout -k 10 200 python -u scripts/filter_bench.py > $O/filter3.txt 2>&1 && cat $O/filter3.txt || { echo bench FAIL; tail -20 $O/filter3.txt; exit 1; }
PBX_FILTER3=0 timeout -k 10 200 python -u scripts/filter_bench.py 2 5 > $O/filter2.txt 2>&1 && cat $O/filter2.txt || { echo bench2 FAIL; tail -20 $O/filter2.txt; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/filter_bench.py 2 5 > $O/prof.log 2>&1 && echo prof ok || { echo prof FAIL; tail -20 $O/prof.log; exit 1; }
grep -i filter $O/prof/run_kernel_stats.csv | cut -c1-200
