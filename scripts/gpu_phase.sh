# Per-phase cycles of k_lz77 / k_huff / k_encode (PBX_PHASE_PROFILE stamps) and the PMC
# passes of the headline workload (issue roofline + traffic), one rocprofv3 pass per counter set.
set -o pipefail
TAG=${1:-phase}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python -u scripts/phase_profile.py noise 4096 > $O/phase_noise.log 2>&1 && cat $O/phase_noise.log || { echo phase FAIL; tail -20 $O/phase_noise.log; exit 1; }
if [ "$2" = "pmc" ]; then
bash scripts/pmc_run.sh > $O/pmc_run.log 2>&1 && echo pmc ok || { echo pmc FAIL; tail -20 $O/pmc_run.log; exit 1; }
mkdir -p $O/pmc && cp -r gpurun_out/pmc[0-9] $O/pmc/ && python3 scripts/pmc_summary.py gpurun_out $O/traffic.json > $O/pmc_summary.txt && tail -80 $O/pmc_summary.txt
if [ -d gpurun_out/pmcf ]; then python3 scripts/pmc_summary.py gpurun_out/pmcf $O/traffic_filter.json > $O/pmc_filter_summary.txt && cat $O/pmc_filter_summary.txt; fi
fi
