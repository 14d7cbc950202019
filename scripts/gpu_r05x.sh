# Round-5: the full GPU suite on the product library, the k_filter3 variants and the
# wave-RLE on/off latency A/B.
set -o pipefail
mkdir -p gpurun_out/r05x
V=$PWD/omero-ms-pixel-buffer_amd/lib
P=$V/libpbx.so
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests > gpurun_out/r05x/pytest_gpu.log 2>&1 || exit 1
PBX_LIB=$V/var_f3c0/libpbx.so timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_sweep.py > gpurun_out/r05x/filt_c0.log 2>&1 || exit 1
PBX_LIB=$V/var_f3nb4/libpbx.so timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_sweep.py > gpurun_out/r05x/filt_nb4.log 2>&1 || exit 1
PBX_LIB=$V/var_sw0/libpbx.so timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_sweep.py > gpurun_out/r05x/filt_sw0.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $P $V/var_f3c0/libpbx.so $V/var_f3nb4/libpbx.so $V/var_sw0/libpbx.so $V/var_f3old/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/filter_bench.py 4 5 || exit 1; done; done > gpurun_out/r05x/filter.log 2>&1 || exit 1
for i in 1 2; do for LL in $P $V/var_rle0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c1_latency.py 2000 2>&1 | grep served || exit 1; done; done > gpurun_out/r05x/c1.log 2>&1 || exit 1
