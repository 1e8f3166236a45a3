#!/bin/bash
# Phase ablation of the split C2 engine: per-launch kernel times of the current
# build and of every _lib_v_* variant (tools/mk_variant.sh ... -DC2_ABL=<mask>),
# every codeword active (tools/c2_ablate.py), two interleaved rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abl; rm -rf $O; mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python tools/c2_ablate.py 256 10 3 >> $O/cur.jsonl 2>> $O/err.log
  for d in ldpc_sparc_amd/_lib_v_abl*; do
    n=${d#ldpc_sparc_amd/_lib_v_}
    LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/c2_ablate.py 256 10 3 >> $O/$n.jsonl 2>> $O/err.log
    echo "$i $n" 
  done
done
echo done
