#!/bin/bash
# R=1.3 (early-stopping) C2 line against the hand-over threshold.
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/ho; mkdir -p gpurun_out/ho
for h in ${HO_LIST:-0.5 0.35 0.2 0.65}; do
  SG_AMP_HANDOVER=$h timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --cpu-seconds 0 --steps 10 > gpurun_out/ho/h_$h.json 2>gpurun_out/ho/h_$h.err
done
