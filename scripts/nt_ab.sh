# Nontemporal loads/stores A/B (one gpurun call): k_extract (raw grid aligned/unaligned,
# configs[3]'s TIFF pass, configs[4]'s pass) for the product (PBX_EXT_NT=3) against
# lib/var_nt0 (=0), and k_filter3 with nontemporal plane loads (lib/var_f3ntl) against the
# product: bash scripts/nt_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
P=omero-ms-pixel-buffer_amd
for i in 1 2; do
  for L in lib/libpbx.so lib/var_nt0/libpbx.so; do
    PBX_LIB=$PWD/$P/$L timeout -k 10 200 python -u scripts/raw_probe.py 5 > $O/raw.log 2>&1 || { tail -20 $O/raw.log; exit 1; }
    echo "$L $(grep -E '^(aligned|unaligned)' $O/raw.log | tr '\n' ' ')"
    PBX_LIB=$PWD/$P/$L timeout -k 10 300 python -u scripts/c4_probe.py > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
    echo "$L c4 $(tail -1 $O/c4.log)"
    PBX_LIB=$PWD/$P/$L timeout -k 10 200 python -u scripts/c5_pass.py 2 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
    echo "$L c5 $(grep 'pass 1' $O/c5.log) $(grep serial $O/c5.log | cut -c1-60)"
  done
  for L in lib/libpbx.so lib/var_f3ntl/libpbx.so; do
    PBX_LIB=$PWD/$P/$L timeout -k 10 300 python -u scripts/filter_bench.py 1 2 4 5 > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
    echo "$L $(cut -c1-62 $O/f.log | tr '\n' '|')"
  done
done
