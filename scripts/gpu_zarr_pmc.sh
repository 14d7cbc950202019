set -o pipefail
mkdir -p gpurun_out/zpmc
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/zpmc/kt -o kt --output-format csv -- python3 scripts/zarr_prof_small.py blosc > gpurun_out/zpmc/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM -d gpurun_out/zpmc/p1 -o p1 --output-format csv -- python3 scripts/zarr_prof_small.py blosc > gpurun_out/zpmc/p1.log 2>&1
