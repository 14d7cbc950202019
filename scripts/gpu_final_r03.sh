# Round-3 final call: parity tests and smoke, the PMC passes of the headline workload (their
# traffic/issue summaries placed under profiles/<TAG>_pmc/ first, so that the bench line's
# roofline cites them), then the bench line and the rocprofv3 kernel-trace summary of it.
# Usage (from the repo root on the box): bash scripts/gpu_final_r03.sh TAG
set -o pipefail
TAG=${1:-final}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_residency.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_residency.log 2>&1 && echo residency ok || { echo residency FAIL; tail -60 $O/pytest_residency.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo tests ok || { echo tests FAIL; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok || { echo smoke FAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 200 python -u scripts/phase_profile.py noise 4096 > $O/phase_noise.log 2>&1 || { echo phase FAIL; tail -20 $O/phase_noise.log; exit 1; }
PMC_FILTER=${PMC_FILTER:-1} bash scripts/pmc_run.sh > $O/pmc_run.log 2>&1 || { echo pmc_run FAIL; tail -20 $O/pmc_run.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out $O/traffic.json > $O/pmc_summary.txt || { echo pmc_summary FAIL; exit 1; }
if [ -d gpurun_out/pmcf ]; then python3 scripts/pmc_summary.py gpurun_out/pmcf $O/traffic_filter.json > $O/pmc_filter_summary.txt || true; fi
cp gpurun_out/pmc0/run_kernel_stats.csv $O/pmc_kernel_stats.csv
mkdir -p profiles/${TAG}_pmc && cp $O/traffic.json $O/issue.json profiles/${TAG}_pmc/
echo pmc ok
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err && echo bench ok || { echo bench FAIL; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
PBX_KSTREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/prof_bench.json 2> $O/prof.log && echo prof ok || { echo prof FAIL; tail -30 $O/prof.log; exit 1; }
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
