#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4t; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_amp_gpu.py -x -v --timeout 200 --timeout-method thread -k c4 > $O/tests.log 2>&1
