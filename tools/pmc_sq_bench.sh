#!/bin/bash
# SQ counters of the bench kernels (every engine the bench line runs: C2 cw2_*,
# f64 cw2d_*, C3 BP, C4 / notebook blk*, C5 GEMM), two passes of at most 8 SQ
# counters each over a short bench run, summarised per kernel by
# tools/pmc_sq_bench.py.  SQ_ARGS overrides the bench arguments, SQ_OUT the
# output directory.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${SQ_OUT:-gpurun_out/sqb}; rm -rf $O; mkdir -p $O
ARGS=${SQ_ARGS:-"--cpu-seconds 0 --no-r13 --bp-ebn0-extra --steps 2 --warmup 1 --bp-steps 3 --sc-steps 1 --concat-steps 1"}
export SQ_ARGS_USED="$ARGS"
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p1 -o run -- python bench.py $ARGS --detail-dir $O > $O/b1.json 2> $O/p1.err
timeout -s KILL 400 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/p2 -o run -- python bench.py $ARGS --detail-dir $O > $O/b2.json 2> $O/p2.err
python tools/pmc_sq_bench.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv $O/sq.json $O/b1.json > $O/sq.log 2>&1
