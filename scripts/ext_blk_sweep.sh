# k_extract's unaligned workgroup size ($PBX_EXT_BLK_UA) on the raw grid at x*bpp mod 16 = 6 and
# on configs[4]'s pass, alternating (one gpurun call): bash scripts/ext_blk_sweep.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do for ub in 16384 24576 32768; do
  PBX_EXT_BLK_UA=$ub timeout -k 10 200 python -u scripts/raw_probe.py 5 > $O/raw.log 2>&1 || { tail -20 $O/raw.log; exit 1; }
  echo "ua_blk=$ub $(grep unaligned $O/raw.log)"
  PBX_EXT_BLK_UA=$ub timeout -k 10 200 python -u scripts/c5_pass.py 2 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
  echo "ua_blk=$ub c5 $(grep 'pass 1' $O/c5.log) $(grep serial $O/c5.log | cut -c1-60)"
done; done
