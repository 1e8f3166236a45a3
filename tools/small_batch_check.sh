#!/bin/bash
# C2 at small batches: default plan (P = 8192 tables, staged engine below one
# wave) against SG_AMP_ENGINE=staged at plan creation (P = 16384).
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/sb; mkdir -p gpurun_out/sb
for B in 32 128; do
  timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 --batch $B --steps 5 > gpurun_out/sb/default_$B.json 2>/dev/null
  SG_AMP_ENGINE=staged timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 --batch $B --steps 5 > gpurun_out/sb/p16k_$B.json 2>/dev/null
done
