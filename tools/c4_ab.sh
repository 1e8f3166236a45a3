#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4ab; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_amp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python tools/c4_ab.py '' general 64 2 > $O/ab.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python tools/c4_ab.py '' '' 64 1 > $O/prof.log 2>&1
