#!/bin/bash
# usage: bash tools/ab_env.sh VAR A B  -- in-process A/B (tools/ab_env.py) plus per-kernel stats of each variant
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_env; rm -rf $O; mkdir -p $O
timeout -k 10 300 python tools/ab_env.py $1 $2 $3 256 4 > $O/ab.log 2>&1
for V in $2 $3; do
  ( export "$1=$V"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks$V -o run -- python tools/amp_c2_probe.py 256 2 1.5 > $O/prof_$V.log 2>&1 )
done
