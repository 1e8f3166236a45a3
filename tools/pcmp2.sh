#!/bin/bash
# P = 16384 (one workgroup per CU) vs P = 8192 (two per CU): probe, kernel stats, tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pcmp2; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_amp_gpu.py -x -q > $O/tests16k.log 2>&1
SG_AMP_PMAX=8192 timeout -k 10 400 python -m pytest tests/test_amp_gpu.py -x -q > $O/tests8k.log 2>&1
for PM in 16384 8192; do
  SG_AMP_PMAX=$PM timeout -k 10 300 python tools/amp_c2_probe.py 256 3 1.5 > $O/probe_$PM.log 2>&1
  SG_AMP_PMAX=$PM timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$PM -o run -- python tools/amp_c2_probe.py 256 2 1.5 > $O/prof_$PM.log 2>&1
done
