# Round-5: all five filters on the product library, the bench line, and k_huff's wave RLE
# (1: both k_huff variants, 2: the batch variant only, 0: off) on c1 latency and the batch.
set -o pipefail
mkdir -p gpurun_out/r05y
V=$PWD/omero-ms-pixel-buffer_amd/lib
timeout -k 10 200 python -u scripts/filter_bench.py > gpurun_out/r05y/filter.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r05y/bench.log 2>&1 || exit 1
for i in 1 2 3; do for LL in $V/libpbx.so $V/var_rle2/libpbx.so $V/var_rle0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/c1_latency.py 3000 2>&1 | grep served || exit 1; done; done > gpurun_out/r05y/c1.log 2>&1 || exit 1
for i in 1 2; do for LL in $V/libpbx.so $V/var_rle0/libpbx.so; do echo "== $LL"; PBX_LIB=$LL timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -1 || exit 1; done; done > gpurun_out/r05y/pw.log 2>&1 || exit 1
