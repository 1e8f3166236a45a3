#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bp; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bp_gpu.py tests/test_pipeline_gpu.py tests/test_integrated_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python tools/bp_quick.py 4096 > $O/quick.log 2>&1
