#!/bin/bash
# Companion-plan change: AMP GPU tests + small/full batch bench lines.
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/cp; mkdir -p gpurun_out/cp
timeout -k 10 600 python -u -m pytest tests/test_amp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cp/tests.log 2>&1
for B in 32 128 256; do
  timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 --batch $B --steps 5 > gpurun_out/cp/b_$B.json 2>gpurun_out/cp/b_$B.err
done
