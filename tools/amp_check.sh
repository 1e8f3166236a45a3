#!/bin/bash
# AMP parity tests + f32 diagnostic + C2 probe with kernel stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/quick; rm -rf $O; mkdir -p $O
timeout -k 10 300 python tools/diag_f32.py > $O/diag.log 2>&1
timeout -k 10 400 python -m pytest tests/test_amp_gpu.py -q > $O/tests.log 2>&1 || true
timeout -k 10 300 python tools/amp_c2_probe.py 256 3 1.5 > $O/probe_generic.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python tools/amp_c2_probe.py 256 2 1.5 > $O/prof.log 2>&1
