#!/bin/bash
# C4 (spatially coupled) probe and kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4; rm -rf $O; mkdir -p $O
timeout -k 10 300 python tools/amp_c4_probe.py 64 2 1.5 > $O/probe.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python tools/amp_c4_probe.py 64 1 1.5 > $O/prof.log 2>&1
