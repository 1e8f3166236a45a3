#!/bin/bash
# Default bench run + rocprofv3 kernel-trace summary of the same command.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bench; rm -rf $O; mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --cpu-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.err
