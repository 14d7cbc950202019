set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01_s5a_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r01_s5a_bench.json 2> gpurun_out/r01_s5a_bench.err
