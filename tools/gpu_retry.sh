#!/bin/bash
# (run from the session host: gpurun with retries only while no box / slot was free -- nothing ran, nothing charged)
# usage: gpu_retry.sh OUTFILE TIMEOUT CMD -- retries only when no box/slot was free (nothing ran)
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  timeout 2400 /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy" $OUT && ! grep -q "status=ok\|status=fail" $OUT; then
    echo "[retry $i] transient, sleeping" >> $OUT.retries; sleep 120; continue
  fi
  break
done
