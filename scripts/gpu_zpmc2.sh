set -o pipefail
mkdir -p gpurun_out/zpmc2
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/zpmc2/kt -o kt --output-format csv -- python3 scripts/zdiag.py > gpurun_out/zpmc2/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d gpurun_out/zpmc2/p1 -o p1 --output-format csv -- python3 scripts/zdiag.py > gpurun_out/zpmc2/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES -d gpurun_out/zpmc2/p2 -o p2 --output-format csv -- python3 scripts/zdiag.py > gpurun_out/zpmc2/p2.log 2>&1
