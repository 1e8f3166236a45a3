#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4skip; rm -rf $O; mkdir -p $O
for K in 0 1 2 3; do
  ( export SG_AMP_SKIP=$K; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks$K -o run -- python tools/c4_ab.py '' '' 64 1 8 > $O/prof$K.log 2>&1 )
done
