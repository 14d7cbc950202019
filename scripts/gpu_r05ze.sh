# Round-5: k_filter3 run length A/B (16 / 32 / 64 rows a wave), k_lz77 phase profile of the
# headline batch, and the PMC passes of the current code (issue + traffic, scripts/pmc_run.sh).
set -o pipefail
mkdir -p gpurun_out/r05ze
V=$PWD/omero-ms-pixel-buffer_amd/lib
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_run16/libpbx.so $V/var_run64/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/filter_bench.py || exit 1; done; done > gpurun_out/r05ze/filter.log 2>&1 || exit 1
PBX_PHASE_PROFILE=1 timeout -k 10 200 python -u scripts/phase_profile.py noise 4096 > gpurun_out/r05ze/phase_noise.log 2>&1 || exit 1
bash scripts/pmc_run.sh > gpurun_out/r05ze/pmc.log 2>&1 || exit 1
