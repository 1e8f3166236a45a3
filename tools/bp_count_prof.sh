#!/bin/bash
# Kernel times of the C3 bench line (rocprofv3 --kernel-trace --stats) for the current build and every
# ldpc_sparc_amd/_lib_v_<name>/: the decode kernel, the error counter and the memsets per step.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bpc; rm -rf $O; mkdir -p $O
A="--no-sc --no-sc-notebook --no-concat --no-r13 --no-f64 --cpu-seconds 0 --bp-ebn0-extra --steps 5"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/base -o run -- python bench.py $A --detail-dir $O/d_base > $O/base.json 2> $O/base.err
for d in ldpc_sparc_amd/_lib_v_*; do
  n=${d#ldpc_sparc_amd/_lib_v_}
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$n -o run -- python bench.py $A --detail-dir $O/d_$n > $O/$n.json 2> $O/$n.err
done
