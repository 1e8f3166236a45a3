#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/streams
for NS in 1 2 4; do
  timeout -k 10 300 python tools/amp_streams_probe.py 256 $NS 3 > gpurun_out/streams/ns$NS.log 2>&1
done
timeout -k 10 300 python tools/amp_streams_probe.py 512 4 3 > gpurun_out/streams/b512ns4.log 2>&1
