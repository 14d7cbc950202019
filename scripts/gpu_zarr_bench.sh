set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u scripts/zarr_bench.py > gpurun_out/r01_s5c_zarr_bench.json 2> gpurun_out/r01_s5c_zarr_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zarr -o zarr --output-format csv -- python3 scripts/zarr_bench.py > gpurun_out/r01_s5c_zarr_prof.log 2>&1
