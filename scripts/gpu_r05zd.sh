# Round-5: k_huff latency changes (second wave for the distance tree, hoisted loads, the
# share check by a wave scan) and k_frame_wave's shorter lane tree: full suite, c1 A/B
# against the previous commit (var_head), phase profile and kernel trace of c1, batch A/B.
set -o pipefail
mkdir -p gpurun_out/r05zd
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zd/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_head/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c1_latency.py 3000 2>&1 | grep served || exit 1; done; done > gpurun_out/r05zd/c1_ab.log 2>&1 || exit 1
PBX_PHASE_PROFILE=1 timeout -k 10 120 python -u scripts/phase_profile.py fake 1 same u8 > gpurun_out/r05zd/phase_c1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05zd/c1prof -o c1 -- python3 -u scripts/c1_latency.py 1000 > gpurun_out/r05zd/c1prof.log 2>&1 || exit 1
for i in 1 2; do for LL in $V/libpbx.so $V/var_head/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -n 2 || exit 1; done; done > gpurun_out/r05zd/pw.log 2>&1 || exit 1
