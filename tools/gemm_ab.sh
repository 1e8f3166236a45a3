#!/bin/bash
# C5 GEMM A/B: tools/gemm_probe.py on the current build and every _lib_v_g* variant, interleaved twice.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gab; rm -rf $O; mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python tools/gemm_probe.py 4 2 >> $O/cur.jsonl 2>> $O/err.log
  for d in ldpc_sparc_amd/_lib_v_g*; do
    n=${d#ldpc_sparc_amd/_lib_v_}
    LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 240 python tools/gemm_probe.py 4 2 >> $O/$n.jsonl 2>> $O/err.log
  done
  echo "round $i"
done
echo done
