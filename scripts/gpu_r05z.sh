# Round-5: k_filter3 bodies per filter (parity + ring depth A/B), then the regression hunt:
# the headline batch (prof_workload noise) on the round-3 final tree, round-4 trees before /
# after the match carry, the round-4 final tree and the current tree, alternating on one box.
set -o pipefail
mkdir -p gpurun_out/r05z
V=$PWD/omero-ms-pixel-buffer_amd/lib
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_lz77.py > gpurun_out/r05z/filt.log 2>&1 || exit 1
for i in 1 2; do for LL in $V/libpbx.so $V/var_nbs8/libpbx.so $V/var_nbs10/libpbx.so $V/var_f3old/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/filter_bench.py || exit 1; done; done > gpurun_out/r05z/filter.log 2>&1 || exit 1
for i in 1 2; do
  for t in _ab/cef8494 _ab/40739cc _ab/b013c52 _ab/0486e88 .; do
    echo "== $t"
    (cd $t && timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -n 3) || exit 1
  done
done > gpurun_out/r05z/ab.log 2>&1
