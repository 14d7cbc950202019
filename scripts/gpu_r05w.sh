# Round-5 experiments: k_huff wave RLE (variant lib) and the k_filter3 rework (product lib).
set -o pipefail
mkdir -p gpurun_out/r05w
L=$PWD/omero-ms-pixel-buffer_amd/lib/var_rlewave/libpbx.so
O=$PWD/omero-ms-pixel-buffer_amd/lib/var_f3old/libpbx.so
C=$PWD/omero-ms-pixel-buffer_amd/lib/var_f3c0/libpbx.so
P=$PWD/omero-ms-pixel-buffer_amd/lib/libpbx.so
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_lz77.py > gpurun_out/r05w/filt.log 2>&1 || exit 1
PBX_LIB=$C timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_sweep.py > gpurun_out/r05w/filt_c0.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $P $C $O; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/filter_bench.py || exit 1; done; done > gpurun_out/r05w/filter.log 2>&1 || exit 1
PBX_LIB=$L timeout -k 10 300 $T tests/test_gpu_huffman.py tests/test_gpu_parity.py tests/test_gpu_sweep.py > gpurun_out/r05w/huff.log 2>&1 || exit 1
PBX_LIB=$L PBX_TIMELINE=1 timeout -k 10 200 python -u scripts/c1_latency.py 2000 > gpurun_out/r05w/c1.log 2>&1 || exit 1
for i in 1 2; do for LL in $P $L; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -1 || exit 1; done; done > gpurun_out/r05w/pw.log 2>&1 || exit 1
