# One GPU call for a change: the GPU parity tests, then the timing workload (deflate stage ms).
# Usage (from the repo root on the box): bash scripts/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo tests ok || { echo tests FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
for g in noise fake; do
  timeout -k 10 120 python scripts/prof_workload.py $g 3 > $O/work_$g.log 2>&1 && tail -1 $O/work_$g.log || { echo work FAIL; tail -20 $O/work_$g.log; exit 1; }
done
