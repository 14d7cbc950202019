# Round-5: k_encode input masking only in the segment's last chunks + bit counts by v_dot4,
# A/B against the previous commit (var_head); the GPU suite first.
set -o pipefail
mkdir -p gpurun_out/r05zg
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zg/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_head/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -n 2 || exit 1; done; done > gpurun_out/r05zg/ab.log 2>&1 || exit 1
