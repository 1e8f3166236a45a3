#!/bin/bash
# f64 C2 probe (B = 256) at hand-over thresholds of the split engine to the staged engine (SG_AMP_HANDOVER:
# active fraction below which the staged engine takes the remaining iterations)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/f64ho; rm -rf $O; mkdir -p $O
for i in 1 2; do
  for h in 0.5 0.35 0.25 0.125 0; do
    echo "handover $h" >> $O/probe.log
    SG_AMP_HANDOVER=$h timeout -k 10 200 python tools/amp_probe.py 256 f64 >> $O/probe.log 2>&1
  done
done
echo done
