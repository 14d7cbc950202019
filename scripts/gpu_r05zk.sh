# Round-5: a single-tile batch framed by k_encode's last workgroup (no k_frame_wave launch):
# full suite, c1 latency A/B against var_fs0 (k_frame_wave), kernel trace of c1.
set -o pipefail
mkdir -p gpurun_out/r05zk
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zk/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3 4; do for LL in $V/libpbx.so $V/var_fs0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c1_latency.py 3000 2>&1 | grep served || exit 1; done; done > gpurun_out/r05zk/c1_ab.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05zk/c1prof -o c1 -- python3 -u scripts/c1_latency.py 1000 > gpurun_out/r05zk/c1prof.log 2>&1 || exit 1
