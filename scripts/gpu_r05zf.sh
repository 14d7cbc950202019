# Round-5: k_encode's last wave joins the CRC (no final barrier) vs the barrier form.
set -o pipefail
mkdir -p gpurun_out/r05zf
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zf/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_lw0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -n 2 || exit 1; done; done > gpurun_out/r05zf/ab.log 2>&1 || exit 1
