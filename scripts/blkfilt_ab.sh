# Huffman block size of row-filtered tiles (PBX_BLK_FILT: 3 and the $AB_LIBS builds): the full bench
# line per library, its adaptive and fixed-filter sections: bash scripts/blkfilt_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for L in lib/libpbx.so ${AB_LIBS:-lib/var_bf6/libpbx.so lib/var_bf11/libpbx.so}; do
  n=$(echo $L | tr / _)
  PBX_LIB=$PWD/omero-ms-pixel-buffer_amd/$L timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/b_$n.json 2> $O/b_$n.err || { tail -20 $O/b_$n.err; exit 1; }
  echo "$L done"
done
