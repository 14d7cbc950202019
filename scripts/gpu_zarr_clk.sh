set -o pipefail
mkdir -p gpurun_out
PBX_LIB=$GRAFT_REPO_ROOT/omero-ms-pixel-buffer_amd/lib_clk/libpbx.so timeout -k 10 120 python -u scripts/zarr_prof_small.py blosc > gpurun_out/r01_s5h_clk.log 2>&1
