# Time library variants built under omero-ms-pixel-buffer_amd/lib/var_*/ (experiments).
set -o pipefail
cd $GRAFT_REPO_ROOT
shopt -s nullglob
for d in omero-ms-pixel-buffer_amd/lib/libpbx.so omero-ms-pixel-buffer_amd/lib/var_*/libpbx.so; do
  for g in ${VARIANT_GENS:-noise fake}; do
    echo "== $d $g"
    PBX_LIB=$PWD/$d timeout -k 10 120 python scripts/prof_workload.py $g 3 2>&1 | tail -1 || exit 1
  done
done
