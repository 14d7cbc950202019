# Round-5: issue counters of the deflate chain on adaptive-filtered G_FAKE (the row-filtered
# k_lz77 variant), two PMC passes, each its own rocprofv3 run (kernel trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zz_pmc
PBX_PW_FILTER=5 PBX_KSTREAMS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/r05zz_pmc/pmc1 -o run --output-format csv -- python3 scripts/prof_workload.py fake 2 > gpurun_out/r05zz_pmc/pmc1.log 2>&1 || exit 1
PBX_PW_FILTER=5 PBX_KSTREAMS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d gpurun_out/r05zz_pmc/pmc2 -o run --output-format csv -- python3 scripts/prof_workload.py fake 2 > gpurun_out/r05zz_pmc/pmc2.log 2>&1 || exit 1
