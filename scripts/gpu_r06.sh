# Round-6 GPU recipe (one gpurun call): bash scripts/gpu_r06.sh TAG STAGE...
#   tests    the -m gpu test files named in $TESTS (default: the round's new ones)
#   gputest  the whole -m gpu suite + smoke
#   probe    sub-batch probe (Infinity Cache lever) and the PNG filter kernels alone
#   ab       alternating A/B of the product library against the variant builds in AB_LIBS
#   rehearse the N-rank bench path, two ranks on one GPU
#   knobs    the headline under other pipelining settings
#   probe3   the sub-batch probe on three kernel streams (sub-batches overlap)
#   fvar     the PNG filter kernels of the var_f3* builds
#   cvar     the deflate chain of the chain variant builds (k_huff one read, k_encode from the plane,
#            k_lz77 without its stream store) next to the product library
#   pmcf     PMC passes of k_filter3 (Sub, Paeth, adaptive): issue + traffic
#   pmc      PMC passes of the headline deflate chain (scripts/pmc_run.sh, filter passes off)
#   parity   the output-parity suites alone
#   kstats   rocprofv3 kernel averages of a short headline run
#   raw      k_extract alone (scripts/raw_probe.py), aligned / unaligned, PBX_EXT_BLK 16-64 KiB
#   hwq      the headline and configs[4] under GPU_MAX_HW_QUEUES 4 / 8 / 16
#   c4       configs[3]'s TIFF pass on one channel (scripts/c4_probe.py), product vs AB_LIBS
#   c1       configs[0]'s served latency (scripts/c1_latency.py), product vs AB_LIBS
#   c5       configs[4]'s pass alone (scripts/c5_pass.py) and its rocprofv3 kernel trace
#   bench    the full bench.py line + the rocprofv3 kernel trace of a serial pass
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
for stage in "$@"; do
  echo "== stage $stage $(date +%T)"
  case $stage in
    tests)
      timeout -k 10 900 $PYT -m gpu ${TESTS:-tests/test_gpu_deflate_scale.py} > $O/pytest_new.log 2>&1 || { grep -E "FAILED|^E " $O/pytest_new.log | head -30; tail -30 $O/pytest_new.log; exit 1; }
      tail -3 $O/pytest_new.log ;;
    gputest)
      timeout -k 10 1000 $PYT -m gpu tests > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|Error" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
      tail -3 $O/pytest_gpu.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    probe)
      timeout -k 10 300 python -u scripts/subbatch_probe.py 5 > $O/subbatch.log 2>&1 || { tail -30 $O/subbatch.log; exit 1; }
      cat $O/subbatch.log | tail -6
      timeout -k 10 300 python -u scripts/filter_bench.py 1 2 3 4 5 > $O/filter.log 2>&1 || { tail -30 $O/filter.log; exit 1; }
      cat $O/filter.log ;;
    lz77)  # the LZ77 parity test alone; its failure is reported, the later stages still run
      timeout -k 10 300 $PYT tests/test_gpu_lz77.py > $O/pytest_lz77.log 2>&1; rc=$?
      [ $rc -eq 124 ] || [ $rc -eq 137 ] && { tail -20 $O/pytest_lz77.log; exit 1; }
      grep -E "^E  |passed|failed" $O/pytest_lz77.log | head -20 ;;
    ab)  # alternating A/B of the product library against variant builds (AB_LIBS: their libpbx.so paths,
         # built beforehand with make OUT=lib/var_<name>; none given: the product library alone)
      for i in 1 2 3; do
        for L in omero-ms-pixel-buffer_amd/lib/libpbx.so ${AB_LIBS:-}; do
          for g in ${AB_GENS:-noise fake}; do
            PBX_LIB=$PWD/$L timeout -k 10 200 python -u scripts/prof_workload.py $g 5 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
            echo "$i $L $(tail -1 $O/ab.log)"
          done
        done
      done ;;
    rehearse)  # the N-rank bench path with both ranks on the box's one GPU (PBX_BENCH_ONE_GPU)
      PBX_BENCH_ONE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/rehearse.json 2> $O/rehearse.err || { tail -30 $O/rehearse.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/rehearse.json')); print(d['n_gpus'], d['value'], sorted(k for k in d if isinstance(d[k], dict))[:40])" ;;
    knobs)  # the headline under other pipelining settings (streams / stagger / depth / sub-batches)
      for kv in "3 1 2 0" "3 1 3 0" "2 1 2 0" "4 1 3 0" "3 2 2 0" "3 0 2 0" "3 1 2 1024" "3 1 4 1024" "4 1 8 512"; do
        set -- $kv
        PBX_KSTREAMS=$1 PBX_KSTAGGER=$2 PBX_BENCH_DEPTH=$3 PBX_BENCH_SUB=$4 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/knob.json 2> $O/knob.err || { tail -20 $O/knob.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/knob.json')); print('streams $1 stagger $2 depth $3 sub $4:', d['value'], d['ms_per_step'])"
      done ;;
    probe3)
      PROBE_KSTREAMS=3 timeout -k 10 300 python -u scripts/subbatch_probe.py 5 > $O/subbatch3.log 2>&1 || { tail -30 $O/subbatch3.log; exit 1; }
      tail -6 $O/subbatch3.log ;;
    fvar)
      for i in 1 2; do for L in omero-ms-pixel-buffer_amd/lib/libpbx.so omero-ms-pixel-buffer_amd/lib/var_f3*/libpbx.so; do
        [ -f "$L" ] || continue
        echo "-- $L"
        PBX_LIB=$PWD/$L timeout -k 10 200 python -u scripts/filter_bench.py ${FILTERS:-1 2 3 4 5} > $O/fvar.log 2>&1 || { tail -20 $O/fvar.log; exit 1; }
        cat $O/fvar.log
      done; done ;;
    cvar)
      for L in omero-ms-pixel-buffer_amd/lib/libpbx.so omero-ms-pixel-buffer_amd/lib/var_*/libpbx.so; do
        case $L in *var_f3*) continue ;; esac
        for g in noise fake; do
          echo "-- $L $g"
          PBX_LIB=$PWD/$L timeout -k 10 200 python -u scripts/prof_workload.py $g 6 > $O/cvar.log 2>&1 || { tail -20 $O/cvar.log; exit 1; }
          tail -2 $O/cvar.log
        done
      done ;;
    pmcf)
      for f in 1 4 5; do
        P=$O/pmcf$f
        mkdir -p $P
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $P/pmc1 -o run --output-format csv -- python3 scripts/filter_bench.py $f > $P/p1.log 2>&1 || { tail -20 $P/p1.log; exit 1; }
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d $P/pmc2 -o run --output-format csv -- python3 scripts/filter_bench.py $f > $P/p2.log 2>&1 || { tail -20 $P/p2.log; exit 1; }
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/pmc3 -o run --output-format csv -- python3 scripts/filter_bench.py $f > $P/p3.log 2>&1 || { tail -20 $P/p3.log; exit 1; }
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/pmc4 -o run --output-format csv -- python3 scripts/filter_bench.py $f > $P/p4.log 2>&1 || { tail -20 $P/p4.log; exit 1; }
        python3 scripts/pmc_summary.py $P $P/traffic.json > $P/summary.txt 2>&1 || true
        grep -A 14 '"k_filter3' $P/summary.txt | head -32
      done ;;
    pmc)
      PMC_FILTER=0 bash scripts/pmc_run.sh > $O/pmc_run.log 2>&1 || { tail -30 $O/pmc_run.log; exit 1; }
      python3 scripts/pmc_summary.py gpurun_out $O/traffic.json > $O/pmc_summary.txt 2>&1 || true
      tail -60 $O/pmc_summary.txt ;;
    parity)  # the output-parity suites (PNG / TIFF bytes against the oracle and the emulator)
      timeout -k 10 400 $PYT tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sweep.py \
        tests/test_gpu_lz77.py tests/test_gpu_huffman.py > $O/pytest_parity.log 2>&1 || { grep -E "FAILED|^E " $O/pytest_parity.log | head -30; tail -5 $O/pytest_parity.log; exit 1; }
      tail -1 $O/pytest_parity.log ;;
    kstats)  # the rocprofv3 kernel averages of a short serial-pass headline run
      PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kprof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline > $O/kprof_bench.json 2> $O/kprof_bench.err || { tail -20 $O/kprof_bench.err; exit 1; }
      find $O/kprof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_short.csv \;
      cut -d, -f1-4 $O/kernel_stats_short.csv | head -12 ;;
    raw)  # k_extract alone, aligned and unaligned, at several workgroup sizes
      for i in 1 2; do for L in omero-ms-pixel-buffer_amd/lib/libpbx.so ${AB_LIBS:-}; do
        for eb in ${EXT_BLKS:-16384 32768 65536}; do
          echo "-- $L"
          PBX_LIB=$PWD/$L PBX_EXT_BLK=$eb timeout -k 10 200 python -u scripts/raw_probe.py 5 > $O/raw.log 2>&1 || { tail -20 $O/raw.log; exit 1; }
          cat $O/raw.log
        done
      done; done ;;
    hwq)  # hardware queues per process (GPU_MAX_HW_QUEUES): the headline and configs[4] at 4 / 8 / 16
      for q in 4 8 16 4 8; do
        GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/hwq.json 2> $O/hwq.err || { tail -20 $O/hwq.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/hwq.json')); print('hwq $q headline', d['value'], d['ms_per_step'], d['kernel_streams']['serial_pass_tiles_per_s'])"
        GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u scripts/c5_pass.py 2 > $O/hwq_c5.log 2>&1 || { tail -20 $O/hwq_c5.log; exit 1; }
        echo "hwq $q c5: $(grep 'pass 1' $O/hwq_c5.log)"
      done ;;
    c4)  # configs[3]'s TIFF pass on one channel, the product library and AB_LIBS, twice
      for i in 1 2; do for L in omero-ms-pixel-buffer_amd/lib/libpbx.so ${AB_LIBS:-}; do
        echo "-- $L"
        PBX_LIB=$PWD/$L timeout -k 10 300 python -u scripts/c4_probe.py > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
        cat $O/c4.log
      done; done ;;
    c1)  # configs[0]'s served single-request latency, product vs AB_LIBS, three alternations
      for i in 1 2 3; do for L in omero-ms-pixel-buffer_amd/lib/libpbx.so ${AB_LIBS:-}; do
        echo "== $L"
        PBX_LIB=$PWD/$L timeout -k 10 200 python -u scripts/c1_latency.py 3000 > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
        grep served $O/c1.log
      done; done ;;
    c5)
      for L in omero-ms-pixel-buffer_amd/lib/libpbx.so ${AB_LIBS:-}; do
        echo "-- $L"
        PBX_LIB=$PWD/$L timeout -k 10 300 python -u scripts/c5_pass.py 3 > $O/c5_pass.log 2>&1 || { tail -20 $O/c5_pass.log; exit 1; }
        cat $O/c5_pass.log
      done
      echo "-- product, PBX_SPLIT_EXTRACT=0"
      PBX_SPLIT_EXTRACT=0 timeout -k 10 300 python -u scripts/c5_pass.py 3 > $O/c5_pass.log 2>&1 || { tail -20 $O/c5_pass.log; exit 1; }
      cat $O/c5_pass.log
      timeout -k 10 300 python -u scripts/c5_pass.py 3 > $O/c5_pass.log 2>&1 || { tail -20 $O/c5_pass.log; exit 1; }
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5prof -o run --output-format csv -- python3 scripts/c5_pass.py 1 > $O/c5_prof.log 2>&1 || { tail -20 $O/c5_prof.log; exit 1; }
      find $O/c5prof -name "*kernel_stats.csv" -exec cp {} $O/c5_kernel_stats.csv \;
      cut -d, -f1-4 $O/c5_kernel_stats.csv | head -16 ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['deflate_chain_ms'], d['roofline']['frac'])"
      PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
      find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \; ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
