#!/bin/bash
# Per-codeword engine tests, and C2 at R=1.3 (early stopping) and R=1.5 on the
# automatic engine choice against the staged engine.
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r13; mkdir -p gpurun_out/r13
timeout -k 10 400 python -u -m pytest tests/test_amp_gpu.py -x -v --timeout 250 --timeout-method thread -k "cw_engine" > gpurun_out/r13/tests.log 2>&1
timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 --rate 1.3 --steps 5 > gpurun_out/r13/auto13.json 2>/dev/null
SG_AMP_ENGINE=staged timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 --rate 1.3 --steps 5 > gpurun_out/r13/staged13.json 2>/dev/null
timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 --steps 5 > gpurun_out/r13/auto15.json 2>/dev/null
