# Headline A/B (one gpurun call): bench.py --no-extra for the product library and each of
# $AB_LIBS (paths under omero-ms-pixel-buffer_amd/), alternating $ROUNDS times (default 3):
# bash scripts/head_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for i in $(seq 1 ${ROUNDS:-3}); do
  for L in lib/libpbx.so ${AB_LIBS:-}; do
    PBX_LIB=$PWD/omero-ms-pixel-buffer_amd/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra > $O/h.json 2> $O/h.err || { tail -20 $O/h.err; exit 1; }
    echo "$L $(python3 scripts/head_summary.py $O/h.json)"
  done
done
