# Diagnostics call: per-phase cycle stamps (PBX_PHASE_PROFILE build path) + the PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/phase_profile.py noise 4096 > gpurun_out/phase_noise.log 2>&1 && echo phase ok || { echo phase FAIL; tail -20 gpurun_out/phase_noise.log; exit 1; }
timeout -k 10 200 python scripts/phase_profile.py fake 4096 > gpurun_out/phase_fake.log 2>&1 && echo phase fake ok || { echo phase FAIL; tail -20 gpurun_out/phase_fake.log; exit 1; }
cat gpurun_out/phase_noise.log gpurun_out/phase_fake.log
bash scripts/pmc_run.sh && python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.txt && cat gpurun_out/pmc_summary.txt
