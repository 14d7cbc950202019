# Round-5: k_lz77's early return for waves with nothing to keep (no reachable boundary), A/B
# against the loop form (var_eo0) and the no-carry timing bound (var_noreach), plus the
# round-3 tree; parity of the product library first.
set -o pipefail
mkdir -p gpurun_out/r05zb
V=$PWD/omero-ms-pixel-buffer_amd/lib
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_lz77.py tests/test_gpu_parity.py tests/test_gpu_huffman.py > gpurun_out/r05zb/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for LL in $V/libpbx.so $V/var_rl0/libpbx.so $V/var_rdisc/libpbx.so $V/var_noreach/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -n 2 || exit 1; done
  echo "== r03"; (cd _ab/cef8494 && timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -n 2) || exit 1
done > gpurun_out/r05zb/ab.log 2>&1 || exit 1
for LL in $V/libpbx.so $V/var_rl0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py fake 3 | tail -n 2 || exit 1; done >> gpurun_out/r05zb/ab.log 2>&1
