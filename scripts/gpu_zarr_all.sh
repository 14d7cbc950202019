set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_zarr.py -m gpu -x -q --timeout 120 --timeout-method thread -s > gpurun_out/r01_s5d_zarr_gpu.log 2>&1 && \
timeout -k 10 300 python -u scripts/zarr_bench.py > gpurun_out/r01_s5d_zarr_bench.json 2> gpurun_out/r01_s5d_zarr_bench.err
