# Round-5: row-start wave-start predictions for row-filtered batches (PBX_LZ_ROWPRED=1, libpbx.so)
# against var_rp0 (the segment-start chain): LZ77 / parity suites (incl. the adaptive-filter
# structured fuzz), then alternating G_FAKE batches with the adaptive / Sub / Up filters and
# adaptive G_NOISE.
set -o pipefail
mkdir -p gpurun_out/r05zw
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lz77.py tests/test_gpu_parity.py > gpurun_out/r05zw/pytest_lz.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_rp0/libpbx.so; do for F in 5 1 2; do
  echo "== $LL filter $F fake"; PBX_LIB=$LL PBX_PW_FILTER=$F timeout -k 10 200 python -u scripts/prof_workload.py fake 5 2>&1 | tail -2 || exit 1
done
  echo "== $LL filter 5 noise"; PBX_LIB=$LL PBX_PW_FILTER=5 timeout -k 10 200 python -u scripts/prof_workload.py noise 5 2>&1 | tail -2 || exit 1
done; done > gpurun_out/r05zw/ab.log 2>&1 || exit 1
