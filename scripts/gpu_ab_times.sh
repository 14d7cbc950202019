# Alternating timing of lib/libpbx.so against lib/var_*/libpbx.so (prof_workload phase times),
# ROUNDS rounds, to separate a small difference from run-to-run noise.
set -o pipefail
TAG=${1:-abtimes}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
shopt -s nullglob
for i in $(seq ${ROUNDS:-4}); do
  for d in omero-ms-pixel-buffer_amd/lib/libpbx.so omero-ms-pixel-buffer_amd/lib/var_*/libpbx.so; do
    n=$(basename $(dirname $d)); [ "$n" = lib ] && n=base
    echo -n "$n " | tee -a $O/times.txt
    PBX_LIB=$PWD/$d PBX_KSTREAMS=1 timeout -k 10 120 python scripts/prof_workload.py ${GEN:-noise} 5 2>&1 | tail -1 | tee -a $O/times.txt || exit 1
  done
done
