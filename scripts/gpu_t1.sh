# One GPU test selection under environment variants.  Usage: bash scripts/gpu_t1.sh TAG SELECTOR "ENV..." ...
set -o pipefail
TAG=$1; SEL=$2; shift 2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u -m pytest "$SEL" -x -q -m gpu --timeout 120 --timeout-method thread > $O/t_$i.log 2>&1; rc=$?
  echo "[$v] rc=$rc $(tail -1 $O/t_$i.log)"
  [ $rc -ge 124 ] && exit 1
done
exit 0
