set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke ok || { echo smoke FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && echo bench ok || { echo bench FAIL; tail -30 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
mkdir -p gpurun_out/prof1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof1.log 2>&1 && echo prof ok || { echo prof FAIL; tail -30 gpurun_out/prof1.log; }
find gpurun_out/prof1 -name "*stats*" | head
