set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_zarr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/zq_test.log 2>&1 && \
timeout -k 10 120 python -u scripts/zarr_bench.py > gpurun_out/zq_pipe.log 2>&1 && \
PBX_INFLATE_1WAVE=1 timeout -k 10 120 python -u scripts/zarr_bench.py > gpurun_out/zq_1wave.log 2>&1 && \
PBX_LIB=$PWD/omero-ms-pixel-buffer_amd/lib/var_zdiag/libpbx.so timeout -k 10 120 python scripts/zdiag.py > gpurun_out/zq_diag.log 2>&1
