# Experimental library variants under lib/var_*/: the profiling workload's kernel times and
# one PMC pass (instruction mix) per variant, summarised per kernel.
set -o pipefail
TAG=${1:-varpmc}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
shopt -s nullglob
timeout -k 10 300 python -u -m pytest ${VTESTS:-tests/test_gpu_lz77.py tests/test_gpu_parity.py} -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && echo tests ok || { echo tests FAIL; tail -30 $O/pytest.log; exit 1; }
for d in omero-ms-pixel-buffer_amd/lib/libpbx.so omero-ms-pixel-buffer_amd/lib/var_*/libpbx.so; do
  n=$(basename $(dirname $d)); [ "$n" = lib ] && n=base
  echo "== $n" | tee -a $O/times.txt
  PBX_LIB=$PWD/$d PBX_KSTREAMS=1 timeout -k 10 120 python scripts/prof_workload.py ${GEN:-noise} 3 2>&1 | tail -1 | tee -a $O/times.txt || exit 1
  PBX_LIB=$PWD/$d PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/p_$n/pmc1 -o run --output-format csv -- python3 scripts/prof_workload.py ${GEN:-noise} 2 > $O/p_$n.log 2>&1 || { echo pmc FAIL; tail -20 $O/p_$n.log; exit 1; }
  python3 scripts/pmc_summary.py $O/p_$n > $O/p_$n.txt && grep -A9 "k_lz77\|k_encode" $O/p_$n.txt | grep -v "^ *\"" | head -24
done
