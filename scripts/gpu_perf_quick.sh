# Quick perf loop: GPU parity of the deflate path + variant timings + phase profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-q}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lz77.py tests/test_gpu_huffman.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && echo tests ok || { echo tests FAIL; tail -40 gpurun_out/$T/pytest.log; exit 1; }
VARIANT_GENS=${VARIANT_GENS:-noise fake} bash scripts/variants.sh > gpurun_out/$T/var.log 2>&1 || { echo var FAIL; tail -20 gpurun_out/$T/var.log; exit 1; }
cat gpurun_out/$T/var.log
timeout -k 10 200 python scripts/phase_profile.py noise 4096 > gpurun_out/$T/phase.log 2>&1 && tail -4 gpurun_out/$T/phase.log
