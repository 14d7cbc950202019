# Round-5: with the row-start predictions, is the walk's VALU candidate form still worth it on
# row-filtered batches?  libpbx.so (VCAND=2) against var_vc0 (scalar loop), alternating.
set -o pipefail
mkdir -p gpurun_out/r05zx
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_vc0/libpbx.so; do for F in 5 1; do
  echo "== $LL filter $F fake"; PBX_LIB=$LL PBX_PW_FILTER=$F timeout -k 10 200 python -u scripts/prof_workload.py fake 5 2>&1 | tail -2 || exit 1
done; done; done > gpurun_out/r05zx/ab.log 2>&1 || exit 1
