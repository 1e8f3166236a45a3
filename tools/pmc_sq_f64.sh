#!/bin/bash
# SQ counters (two passes of 8) over one f64 C2 probe decode (B = 256), per kernel:
# tools/pmc_sq_bench.py summary in gpurun_out/sqd/sq_summary.txt.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sqd; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p1 -o run -- python tools/amp_c2_probe.py 256 1 1.5 f64 > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/p2 -o run -- python tools/amp_c2_probe.py 256 1 1.5 f64 > $O/p2.log 2>&1
python tools/pmc_sq_bench.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv $O/sq.json cw2d reg_ > $O/sq_summary.txt
echo done
