set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo tests ok || { echo tests FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 200 python scripts/phase_profile.py noise 4096 > gpurun_out/phase_noise.log 2>&1 && echo phase ok || { echo phase FAIL; tail -20 gpurun_out/phase_noise.log; exit 1; }
cat gpurun_out/phase_noise.log
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && echo bench ok || { echo bench FAIL; tail -30 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
