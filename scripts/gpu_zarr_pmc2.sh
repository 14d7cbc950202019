set -o pipefail
mkdir -p gpurun_out/zpmc2
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_zarr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/zpmc2/pytest.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/zpmc2/f -o f --output-format csv -- python3 scripts/zarr_prof_small.py blosc > gpurun_out/zpmc2/f.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/zpmc2/w -o w --output-format csv -- python3 scripts/zarr_prof_small.py blosc > gpurun_out/zpmc2/w.log 2>&1
