#!/bin/bash
# Notebook geometry (L = 2048) and C4 (L = 1024): two-position-table form (current build) against the one-table
# form (_lib_v_b2one: -DB2_ONETABLE=1), interleaved, decode probe (tools/amp_c4_probe.py B reps R L)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/b2one; rm -rf $O; mkdir -p $O
for i in 1 2; do
  for L in 2048 1024; do
    echo "cur L=$L" >> $O/probe.log
    timeout -k 10 200 python tools/amp_c4_probe.py 256 3 1.5 $L >> $O/probe.log 2>&1
    echo "b2one L=$L" >> $O/probe.log
    LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_v_b2one/libldpc_sparc_amd.so timeout -k 10 200 python tools/amp_c4_probe.py 256 3 1.5 $L >> $O/probe.log 2>&1
  done
done
echo done
