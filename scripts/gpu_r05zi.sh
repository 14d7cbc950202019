# Round-5: k_filter3 16-row runs for Avg / Paeth (product) vs 32 (var_ap32); parity first.
set -o pipefail
mkdir -p gpurun_out/r05zi
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_lz77.py > gpurun_out/r05zi/tests.log 2>&1 || exit 1
for i in 1 2 3 4; do for LL in $V/libpbx.so $V/var_ap32/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/filter_bench.py 3 4 || exit 1; done; done > gpurun_out/r05zi/filter_ap.log 2>&1 || exit 1
