#!/bin/bash
# After a stage-1 kernel change: phase profile, C2 probe, per-kernel times,
# AMP GPU tests, f32 diagnostics.  Summary: python tools/amp_check_report.py
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/check; rm -rf $O; mkdir -p $O
timeout -k 10 300 python tools/amp_tprof.py 256 > $O/tprof.log 2>&1
timeout -k 10 300 python tools/amp_c2_probe.py 256 3 1.5 > $O/probe.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python tools/amp_c2_probe.py 256 2 1.5 > $O/prof.log 2>&1
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -m pytest tests/test_amp_gpu.py -q -x > $O/tests.log 2>&1
  timeout -k 10 300 python tools/diag_f32.py > $O/diag.log 2>&1
fi
