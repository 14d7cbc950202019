# Adaptive tile mode (k_adaptive_mode) checks in one gpurun call: the adaptive parity tests,
# the adaptive filter kernels A/B against the previous library (var/libpbx_head.so), the
# headline A/B, and the full bench line (its adaptive Poisson bytes): bash scripts/ab_adaptive.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_deflate_scale.py tests/test_gpu_unaligned.py tests/test_gpu_parity.py tests/test_gpu_sweep.py \
  > $O/t.log 2>&1 || { grep -E "FAILED|^E " $O/t.log | head -20; exit 1; }
tail -1 $O/t.log
for i in 1 2; do for L in omero-ms-pixel-buffer_amd/lib/libpbx.so var/libpbx_head.so; do
  PBX_LIB=$PWD/$L timeout -k 10 200 python -u scripts/filter_bench.py 5 > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
  echo "$L $(grep adaptive $O/f.log)"
  PBX_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra > $O/h.log 2>&1 || { tail -20 $O/h.log; exit 1; }
  echo "$L $(tail -1 $O/h.log | cut -c1-160)"
done; done
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
