#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes of the C2 probe (B=256, 1 rep) for tools/pmc_traffic.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc; rm -rf $O; mkdir -p $O
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python tools/amp_c2_probe.py 256 1 1.5 $O/probe_f.json > $O/f.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python tools/amp_c2_probe.py 256 1 1.5 $O/probe_w.json > $O/w.log 2>&1
python tools/pmc_traffic.py $O/f/run_counter_collection.csv $O/w/run_counter_collection.csv $O/probe_f.json $O/traffic.json > $O/traffic.log 2>&1
