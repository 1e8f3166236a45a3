#!/bin/bash
# Quick check: AMP GPU tests, C2 probe (generic and hot stage-1 kernels), kernel stats, LDS counters.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/quick; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_amp_gpu.py -x -q > $O/tests.log 2>&1
SG_AMP_NOHOT=1 timeout -k 10 300 python tools/amp_c2_probe.py 256 3 1.5 > $O/probe_generic.log 2>&1
timeout -k 10 300 python tools/amp_c2_probe.py 256 3 1.5 > $O/probe_hot.log 2>&1
SG_AMP_NOHOT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python tools/amp_c2_probe.py 256 2 1.5 > $O/prof.log 2>&1
SG_AMP_NOHOT=1 timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc -o run -- python tools/amp_c2_probe.py 256 1 1.5 > $O/pmc.log 2>&1
