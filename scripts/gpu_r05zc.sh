# Round-5: full GPU suite on the product library, the bench line, a kernel trace and phase
# profile of the single-request (c1) path, and k_huff's second wave on/off for c1.
set -o pipefail
mkdir -p gpurun_out/r05zc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
PBX_LIB=$V/var_hw1/libpbx.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sweep.py > gpurun_out/r05zc/sweep_hw1.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zc/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_hw1/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c1_latency.py 3000 2>&1 | grep served || exit 1; done; done > gpurun_out/r05zc/c1_ab.log 2>&1 || exit 1
PBX_PHASE_PROFILE=1 timeout -k 10 120 python -u scripts/phase_profile.py fake 1 same u8 > gpurun_out/r05zc/phase_c1.log 2>&1 || exit 1
PBX_LIB=$V/var_hw1/libpbx.so PBX_PHASE_PROFILE=1 timeout -k 10 120 python -u scripts/phase_profile.py fake 1 same u8 > gpurun_out/r05zc/phase_c1_hw1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05zc/c1prof -o c1 -- python3 -u scripts/c1_latency.py 1000 > gpurun_out/r05zc/c1prof.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r05zc/bench.log 2>&1 || exit 1
