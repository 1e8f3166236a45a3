#!/bin/bash
# Texture-address / L1 counters for the C2 AMP decode (vector-memory pipe pressure).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ta; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum --output-format csv -d $O/p1 -o run -- python tools/amp_c2_probe.py 256 1 1.5 > $O/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $O/p2 -o run -- python tools/amp_c2_probe.py 256 1 1.5 > $O/p2.log 2>&1
