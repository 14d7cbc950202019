# Variant A/B on two generators: the deflate parity tests on the product library, then the
# profiling workload (noise, fake) for it and every lib/var_*/ build, one PMC instruction pass
# on noise each.  Usage (on the box): bash scripts/gpu_ab2.sh TAG
set -o pipefail
TAG=${1:-ab2}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest ${VTESTS:-tests/test_gpu_lz77.py tests/test_gpu_parity.py tests/test_gpu_sweep.py} -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && echo tests ok || { echo tests FAIL; tail -30 $O/pytest.log; exit 1; }
shopt -s nullglob
for d in omero-ms-pixel-buffer_amd/lib/libpbx.so omero-ms-pixel-buffer_amd/lib/var_*/libpbx.so; do
  n=$(basename $(dirname $d)); [ "$n" = lib ] && n=base
  for g in noise fake; do
    echo "== $n $g" >> $O/times.txt
    PBX_LIB=$PWD/$d PBX_KSTREAMS=1 timeout -k 10 120 python scripts/prof_workload.py $g 4 2>&1 | tail -2 >> $O/times.txt || exit 1
  done
done
cat $O/times.txt
