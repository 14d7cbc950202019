# Round-5: configs[2] batch and the headline batch, VALU-candidate walk vs var_vc0, alternating.
set -o pipefail
mkdir -p gpurun_out/r05zs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_vc0/libpbx.so; do
  echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c3_probe.py 5 2>&1 | tail -3 || exit 1
  PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 6 2>&1 | tail -3 || exit 1
done; done > gpurun_out/r05zs/ab.log 2>&1 || exit 1
