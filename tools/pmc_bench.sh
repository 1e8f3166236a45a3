#!/bin/bash
# HBM bytes per launch of every bench kernel: rocprofv3 --pmc FETCH_SIZE and
# --pmc WRITE_SIZE in separate passes over a short bench run (no CPU baseline,
# no C5), summarised per kernel by tools/pmc_bench.py with the units of the
# bench line printed by the same run.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmcb; rm -rf $O; mkdir -p $O
ARGS="--cpu-seconds 0 --no-concat --no-r13 --no-f64 --bp-ebn0-extra --steps 3 --warmup 1 --bp-steps 3 --sc-steps 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python bench.py $ARGS --detail-dir $O > $O/bench_f.json 2> $O/f.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python bench.py $ARGS --detail-dir $O > $O/bench_w.json 2> $O/w.err
python tools/pmc_bench.py $O/f/run_counter_collection.csv $O/w/run_counter_collection.csv $O/bench_f.json $O/traffic.json > $O/traffic.log 2>&1
