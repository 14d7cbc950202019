set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_zarr.py -m gpu -x -q --timeout 120 --timeout-method thread -k "strategies or inflate or zlib" > gpurun_out/zt_test.log 2>&1
