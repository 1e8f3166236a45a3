#!/bin/bash
# retry a gpurun call while no box/slot is free (exit 3: nothing ran, nothing charged)
out=$1; shift
for i in $(seq 1 20); do
  timeout 3000 /usr/local/graft/bin/gpurun --timeout 1800 -- "$@" > $out 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "nothing was charged" $out; then break; fi
  sleep 150
done
echo "rc=$rc tries=$i" >> $out
