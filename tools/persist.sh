#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/persist; rm -rf $O; mkdir -p $O
SG_AMP_PERSIST=1 timeout -k 10 400 python -m pytest tests/test_amp_gpu.py -x -q > $O/tests.log 2>&1
for P in 0 1; do
  SG_AMP_PERSIST=$P timeout -k 10 300 python tools/amp_c2_probe.py 256 3 1.5 > $O/probe_$P.log 2>&1
  SG_AMP_PERSIST=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$P -o run -- python tools/amp_c2_probe.py 256 2 1.5 > $O/prof_$P.log 2>&1
done
