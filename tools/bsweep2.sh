#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bsweep; rm -rf $O; mkdir -p $O
for B in 32 64 128 256; do
  timeout -k 10 300 python tools/amp_c2_probe.py $B 3 1.5 > $O/b$B.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks32 -o run -- python tools/amp_c2_probe.py 32 2 1.5 > $O/prof32.log 2>&1
