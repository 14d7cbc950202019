set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_zarr.py -m gpu -x -v --timeout 120 --timeout-method thread -s > gpurun_out/r01_s5b_zarr_gpu.log 2>&1
