# Round 3: all GPU tests, then the filter kernels alone, then the served path (coalescer
# depth x completer threads sweep).
set -o pipefail
TAG=${1:-r03b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo tests ok || { echo tests FAIL; tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -u scripts/filter_bench.py > $O/filter3.txt 2>&1 && cat $O/filter3.txt || { echo filter FAIL; tail -20 $O/filter3.txt; exit 1; }
for nc in 1 2; do
PBX_COMPLETERS=$nc timeout -k 10 300 python -u scripts/serve_sweep.py 3,4 > $O/serve_c$nc.json 2> $O/serve_c$nc.err && echo "completers $nc" && cat $O/serve_c$nc.json || { echo serve FAIL; tail -20 $O/serve_c$nc.err; exit 1; }
done
VARIANT_GENS=noise timeout -k 10 400 bash scripts/variants.sh > $O/variants.txt 2>&1 && cat $O/variants.txt || { echo variants FAIL; tail -20 $O/variants.txt; exit 1; }
