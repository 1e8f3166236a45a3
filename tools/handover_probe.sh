#!/bin/bash
# R = 1.3 C2 probe (tools/amp_c2_probe.py 256 4 1.3) against the hand-over threshold (SG_AMP_HANDOVER), two runs.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ho2
for r in 1 2; do for h in 0.65 0.5 0.35 0.2 0.0; do
  echo "h=$h run=$r" >> gpurun_out/ho2/out.txt
  SG_AMP_HANDOVER=$h timeout -k 10 150 python tools/amp_c2_probe.py 256 4 1.3 >> gpurun_out/ho2/out.txt 2>&1
done; done
