#!/bin/bash
# C2 decode split over NS concurrent streams (tools/amp_streams_probe.py)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/streams
for cfg in ${CFGS:-"256 1" "256 2" "256 4" "512 2"}; do
  set -- $cfg
  timeout -k 10 300 python tools/amp_streams_probe.py $1 $2 3 > gpurun_out/streams/b$1ns$2.log 2>&1
done
