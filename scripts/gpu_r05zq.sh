# Round-5: k_lz77's walk with the candidate lengths in VALU (lane c: candidate c; PBX_LZ_VCAND=1)
# against var_vc0 (the scalar loop): LZ77 parity suites, then alternating timing on G_FAKE with
# the adaptive filter, plain G_FAKE and G_NOISE.
set -o pipefail
mkdir -p gpurun_out/r05zq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lz77.py tests/test_gpu_parity.py > gpurun_out/r05zq/pytest_lz.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_vc0/libpbx.so; do for F in 5 0; do for G in fake noise; do
  [ $F = 5 ] && [ $G = noise ] && continue
  echo "== $LL filter $F $G"; PBX_LIB=$LL PBX_PW_FILTER=$F timeout -k 10 200 python -u scripts/prof_workload.py $G 6 2>&1 | tail -3 || exit 1
done; done; done; done > gpurun_out/r05zq/ab.log 2>&1 || exit 1
