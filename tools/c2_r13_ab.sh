#!/bin/bash
# C2 probe at R = 1.3 (12-14 outputs per thread) and R = 1.5: current build against the _lib_v_c2* variants
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c2r13; rm -rf $O; mkdir -p $O
for i in 1 2; do
  for R in 1.3 1.5; do
    echo "cur R=$R" >> $O/probe.log
    timeout -k 10 120 python tools/amp_c2_probe.py 256 3 $R >> $O/probe.log 2>&1
    for d in ldpc_sparc_amd/_lib_v_c2*; do
      [ -d "$d" ] || continue
      echo "${d#ldpc_sparc_amd/_lib_v_} R=$R" >> $O/probe.log
      LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/amp_c2_probe.py 256 3 $R >> $O/probe.log 2>&1
    done
  done
done
echo done
