#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/stagger; rm -rf $O; mkdir -p $O
for S in 0 10000 20000 30000; do
  SG_AMP_STAGGER=$S timeout -k 10 300 python tools/amp_c2_probe.py 256 3 1.5 > $O/s$S.log 2>&1
done
