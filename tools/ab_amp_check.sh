#!/bin/bash
# AMP GPU parity tests on the current build, then the same-box A/B of the
# current build against every ldpc_sparc_amd/_lib_v_<name>/ (tools/ab_multi.sh).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t1
timeout -k 10 400 python -u -m pytest tests/test_amp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1/amp_tests.log 2>&1
bash tools/ab_multi.sh
