#!/bin/bash
# AMP GPU tests, in-process A/B of an env knob, phase timestamps of both variants
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_amp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python tools/ab_env.py $1 $2 $3 256 3 > $O/ab.log 2>&1
for V in $2 $3; do
  ( export "$1=$V"; timeout -k 10 300 python tools/amp_tprof.py 256 > $O/tprof_$V.log 2>&1 )
done
