#!/bin/bash
# GPU parity suite, smoke, the default bench line and its rocprofv3
# kernel-trace summary.  Stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/full; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --cpu-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.err
