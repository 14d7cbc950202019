# PMC passes over the profiling workload (each pass its own rocprofv3 run, kernel trace
# only; never combined with sys/runtime traces).  Output under gpurun_out/pmc*/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc0 -o run --output-format csv -- python3 scripts/prof_workload.py noise 3 > gpurun_out/pmc0.log 2>&1 || { echo pass0 FAIL; tail -20 gpurun_out/pmc0.log; exit 1; }
PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc1 -o run --output-format csv -- python3 scripts/prof_workload.py noise 2 > gpurun_out/pmc1.log 2>&1 || { echo pass1 FAIL; tail -20 gpurun_out/pmc1.log; exit 1; }
PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc2 -o run --output-format csv -- python3 scripts/prof_workload.py noise 2 > gpurun_out/pmc2.log 2>&1 || { echo pass2 FAIL; tail -20 gpurun_out/pmc2.log; exit 1; }
PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc3 -o run --output-format csv -- python3 scripts/prof_workload.py noise 2 > gpurun_out/pmc3.log 2>&1 || { echo pass3 FAIL; tail -20 gpurun_out/pmc3.log; exit 1; }
PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc4 -o run --output-format csv -- python3 scripts/prof_workload.py noise 2 > gpurun_out/pmc4.log 2>&1 || { echo pass4 FAIL; tail -20 gpurun_out/pmc4.log; exit 1; }
echo all passes ok
find gpurun_out/pmc* -name "*.csv" | head -30
# the PNG filter kernel (k_filter3: Sub = fixed, adaptive), filter_bench's 4096 tiles, its own dir
if [ "${PMC_FILTER:-1}" = "1" ]; then
mkdir -p gpurun_out/pmcf
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmcf/pmc1 -o run --output-format csv -- python3 scripts/filter_bench.py 1 5 > gpurun_out/pmcf1.log 2>&1 || { echo passf1 FAIL; tail -20 gpurun_out/pmcf1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmcf/pmc2 -o run --output-format csv -- python3 scripts/filter_bench.py 1 5 > gpurun_out/pmcf2.log 2>&1 || { echo passf2 FAIL; tail -20 gpurun_out/pmcf2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmcf/pmc3 -o run --output-format csv -- python3 scripts/filter_bench.py 1 5 > gpurun_out/pmcf3.log 2>&1 || { echo passf3 FAIL; tail -20 gpurun_out/pmcf3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmcf/pmc4 -o run --output-format csv -- python3 scripts/filter_bench.py 1 5 > gpurun_out/pmcf4.log 2>&1 || { echo passf4 FAIL; tail -20 gpurun_out/pmcf4.log; exit 1; }
echo filter passes ok
fi
