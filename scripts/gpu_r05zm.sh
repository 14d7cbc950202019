# Round-5: k_huff merge rounds with both rank searches in one branch-free loop, against var_ds0
# var_ds0 (a wave_sum per segment): full suite, c1 phase stamps, c1 latency and batch A/B.
set -o pipefail
mkdir -p gpurun_out/r05zm
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zm/pytest_gpu.log 2>&1 || exit 1
for LL in $V/libpbx.so $V/var_ds0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL PBX_PHASE_PROFILE=1 timeout -k 10 120 python -u scripts/phase_profile.py fake 1 same u8 2>&1 || exit 1; done > gpurun_out/r05zm/phase_c1.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_ds0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c1_latency.py 3000 2>&1 | grep served || exit 1; done; done > gpurun_out/r05zm/c1_ab.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_ds0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 10 2>&1 || exit 1; done; done > gpurun_out/r05zm/batch_ab.log 2>&1 || exit 1
