#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c5; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_campaign_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python tools/c5_sweep.py --codewords 1024 --ebn0 1 2 3 4 5 6 --npz $O/c5.npz > $O/sweep.log 2>&1
