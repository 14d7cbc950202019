# Round-5: the walk's VALU candidate form only in run-dense waves (PBX_LZ_VCAND=2, libpbx.so)
# against always (var_vc1) and never (var_vc0): LZ77 parity, then configs[2], G_NOISE, G_FAKE and
# adaptive-filter G_FAKE batches, alternating.
set -o pipefail
mkdir -p gpurun_out/r05zt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lz77.py tests/test_gpu_parity.py > gpurun_out/r05zt/pytest_lz.log 2>&1 || exit 1
for i in 1 2; do for LL in $V/libpbx.so $V/var_vc1/libpbx.so $V/var_vc0/libpbx.so; do
  echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c3_probe.py 4 2>&1 | tail -2 || exit 1
  PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 5 2>&1 | tail -2 || exit 1
  PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py fake 5 2>&1 | tail -2 || exit 1
  PBX_LIB=$LL PBX_PW_FILTER=5 timeout -k 10 200 python -u scripts/prof_workload.py fake 5 2>&1 | tail -2 || exit 1
done; done > gpurun_out/r05zt/ab.log 2>&1 || exit 1
