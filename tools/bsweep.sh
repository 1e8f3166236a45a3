#!/bin/bash
# C2 AMP decode throughput vs batch size (MALL residency of the row buffer).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bsweep
for B in ${BS:-32 64 128 256}; do
  timeout -k 10 300 python tools/amp_c2_probe.py $B 3 1.5 > gpurun_out/bsweep/b$B.log 2>&1
done
