# Round-5: k_huff's segment bit counts by one transposing butterfly (lane k: segment k) against
# var_ls0 (a wave_sum per segment): full suite, c1 phase stamps, c1 latency and batch A/B.
set -o pipefail
mkdir -p gpurun_out/r05zl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zl/pytest_gpu.log 2>&1 || exit 1
for LL in $V/libpbx.so $V/var_ls0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL PBX_PHASE_PROFILE=1 timeout -k 10 120 python -u scripts/phase_profile.py fake 1 same u8 2>&1 || exit 1; done > gpurun_out/r05zl/phase_c1.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_ls0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c1_latency.py 3000 2>&1 | grep served || exit 1; done; done > gpurun_out/r05zl/c1_ab.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_ls0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 10 2>&1 || exit 1; done; done > gpurun_out/r05zl/batch_ab.log 2>&1 || exit 1
