# Round-5: k_lz77's boundary test for rows <= 256 bytes (a 3-byte row-up run): the new test on
# the previous commit (expected red for run=3), the fixed product and the mask-based variant
# (var_rmask); then the full suite on the product and the product / var_rmask timing.
set -o pipefail
mkdir -p gpurun_out/r05zj
V=$PWD/omero-ms-pixel-buffer_amd/lib
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
PBX_LIB=$V/var_head/libpbx.so timeout -k 10 200 $T tests/test_gpu_lz77.py -k short_rowup > gpurun_out/r05zj/head_short.log 2>&1
echo "head rc=$?" >> gpurun_out/r05zj/head_short.log
PBX_LIB=$V/var_rmask/libpbx.so timeout -k 10 300 $T -x tests/test_gpu_lz77.py tests/test_gpu_parity.py tests/test_gpu_sweep.py > gpurun_out/r05zj/rmask.log 2>&1 || exit 1
timeout -k 10 600 $T -x -m gpu tests > gpurun_out/r05zj/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_rmask/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -n 2 || exit 1; done; done > gpurun_out/r05zj/ab.log 2>&1 || exit 1
for LL in $V/libpbx.so $V/var_rmask/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py fake 3 | tail -n 2 || exit 1; done >> gpurun_out/r05zj/ab.log 2>&1 || exit 1
