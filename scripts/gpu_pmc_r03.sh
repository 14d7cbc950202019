# Round 3: variant A/B (times + one instruction-mix PMC pass each, scripts/gpu_varpmc.sh),
# then the full PMC passes of the product library (scripts/pmc_run.sh) and their summary.
set -o pipefail
TAG=${1:-pmc}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_varpmc.sh $TAG || exit 1
PMC_FILTER=${PMC_FILTER:-0} bash scripts/pmc_run.sh > gpurun_out/$TAG/pmc_run.log 2>&1 || { echo pmc_run FAIL; tail -20 gpurun_out/$TAG/pmc_run.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out gpurun_out/$TAG/traffic.json > gpurun_out/$TAG/pmc_summary.txt && grep -A16 "k_lz77\|k_encode\|k_huff" gpurun_out/$TAG/pmc_summary.txt | head -60
