# PMC passes of the product library (scripts/pmc_run.sh: kernel trace, instruction mix, issue
# and wait counters, FETCH_SIZE, WRITE_SIZE, each its own rocprofv3 run) + the phase stamps.
# Usage (on the box): bash scripts/gpu_pmc_final.sh TAG
set -o pipefail
TAG=${1:-pmc}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 200 python -u scripts/phase_profile.py noise 4096 > gpurun_out/$TAG/phase_noise.log 2>&1 || { echo phase FAIL; tail -20 gpurun_out/$TAG/phase_noise.log; exit 1; }
tail -4 gpurun_out/$TAG/phase_noise.log
PMC_FILTER=${PMC_FILTER:-0} bash scripts/pmc_run.sh > gpurun_out/$TAG/pmc_run.log 2>&1 || { echo pmc_run FAIL; tail -20 gpurun_out/$TAG/pmc_run.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out gpurun_out/$TAG/traffic.json > gpurun_out/$TAG/pmc_summary.txt && grep -A16 "k_lz77\|k_encode" gpurun_out/$TAG/pmc_summary.txt | head -40
cp gpurun_out/pmc0/run_kernel_stats.csv gpurun_out/$TAG/kernel_stats.csv
