# k_adaptive_mode threads per tile (PBX_AM_NT 256 / 128 / 64): the Poisson tile-mode parity test
# and a rocprofv3 kernel trace of filter_bench's adaptive pass per library: bash scripts/am_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
P=omero-ms-pixel-buffer_amd
for L in lib/libpbx.so lib/var_am128/libpbx.so lib/var_am64/libpbx.so; do
  n=$(echo $L | tr / _)
  PBX_LIB=$PWD/$P/$L timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_deflate_scale.py::test_adaptive_tile_mode_poisson > $O/t_$n.log 2>&1 || { tail -20 $O/t_$n.log; exit 1; }
  PBX_LIB=$PWD/$P/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$n -o run -- python3 scripts/filter_bench.py 5 > $O/f_$n.log 2>&1 || { tail -20 $O/f_$n.log; exit 1; }
  echo "$L $(tail -1 $O/t_$n.log) $(grep adaptive $O/f_$n.log | cut -c1-40)"
done
