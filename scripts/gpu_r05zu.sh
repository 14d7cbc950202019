# Round-5: k_lz77<.., VC> -- the walk's VALU candidate form only in row-filtered batches
# (libpbx.so) against var_vc0 (never): the -m gpu suite, then configs[2], G_NOISE, G_FAKE and
# adaptive-filter G_FAKE batches, alternating.
set -o pipefail
mkdir -p gpurun_out/r05zu
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zu/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_vc0/libpbx.so; do
  echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c3_probe.py 4 2>&1 | tail -2 || exit 1
  PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 5 2>&1 | tail -2 || exit 1
  PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py fake 5 2>&1 | tail -2 || exit 1
  PBX_LIB=$LL PBX_PW_FILTER=5 timeout -k 10 200 python -u scripts/prof_workload.py fake 5 2>&1 | tail -2 || exit 1
done; done > gpurun_out/r05zu/ab.log 2>&1 || exit 1
