#!/bin/bash
# Per-codeword engine: AMP parity tests, then the C2 bench line on both engines.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cw; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_amp_gpu.py -x -v --timeout 200 --timeout-method thread -k "cw_engine" > $O/tests.log 2>&1
SG_AMP_ENGINE=cw timeout -k 10 100 python tools/cw_tprof.py > $O/tprof.txt 2>&1
SG_AMP_ENGINE=cw timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 > $O/bench_cw.json 2> $O/bench_cw.err
