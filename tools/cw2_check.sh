#!/bin/bash
# Split per-codeword engine: parity tests, then the C2 probe (B = 256) with the
# split engine (default) and the one-workgroup engine (SG_AMP_CW2=0), same box,
# then the bench line.  Stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cw2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_amp_cw2_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 120 python tools/amp_c2_probe.py 256 6 > $O/probe_cw2.log 2>&1
timeout -k 10 120 env SG_AMP_CW2=0 python tools/amp_c2_probe.py 256 6 > $O/probe_cw1.log 2>&1
timeout -k 10 120 python tools/amp_c2_probe.py 256 6 > $O/probe_cw2b.log 2>&1
timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 --steps 10 > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python -u -m pytest tests/test_amp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/amp_tests.log 2>&1
echo done
