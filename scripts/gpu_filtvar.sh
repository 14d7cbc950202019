# k_filter3 variants: the PNG filter parity tests on the product library, then the filter
# kernels' timing for it and for each experimental build under lib/var_*/.
set -o pipefail
TAG=${1:-filtvar}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 200 --timeout-method thread -k "filter or adaptive or sweep" > $O/pytest_filter.log 2>&1 && echo filter tests ok || { echo filter tests FAIL; tail -40 $O/pytest_filter.log; exit 1; }
shopt -s nullglob
for d in omero-ms-pixel-buffer_amd/lib/libpbx.so omero-ms-pixel-buffer_amd/lib/var_*/libpbx.so; do
  echo "== $d" | tee -a $O/filter3.txt
  PBX_LIB=$PWD/$d timeout -k 10 200 python -u scripts/filter_bench.py ${FILTERS:-} >> $O/filter3.txt 2>&1 || { echo bench FAIL; tail -20 $O/filter3.txt; exit 1; }
done
cat $O/filter3.txt
