#!/bin/bash
# (host side, not run on the box) try a gpurun call when the pool has a box: retries ONLY while gpurun reports no free box /
# backoff (nothing ran, nothing charged); any call that ran is final.
OUT=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout 1500 -- "$@" > $OUT 2>&1
  rc=$?
  if grep -q "backing off" $OUT; then
    s=$(grep -o "retry in [0-9]*s" $OUT | grep -o "[0-9]*" | head -1); sleep $(( ${s:-300} + 5 )); continue
  fi
  if [ $rc -eq 3 ] || grep -q -e "no free box" -e "slot(s) on this pod are busy" -e "retry in a few minutes" -e "stopped responding while being prepared" $OUT; then sleep 240; continue; fi
  echo "attempt $i rc=$rc" >> $OUT
  exit 0
done
