set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_zarr.py -m gpu -x -q --timeout 120 --timeout-method thread -s > gpurun_out/r01_s5e_zarr_gpu.log 2>&1 && \
timeout -k 10 120 python -u scripts/zarr_prof_small.py blosc zlib > gpurun_out/r01_s5e_small.log 2>&1
