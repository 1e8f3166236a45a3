#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tprof; rm -rf $O; mkdir -p $O
for W in 1 0; do
  SG_AMP_WAVEFFT=$W timeout -k 10 300 python tools/amp_tprof.py 256 > $O/tprof_$W.log 2>&1
done
