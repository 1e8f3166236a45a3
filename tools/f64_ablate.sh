#!/bin/bash
# Phase ablation of the f64 split engine: per-launch kernel times of the current build and of every
# _lib_v_d* variant (tools/mk_variant.sh d<mask> amp_cw2d.hip -DD_ABL=<mask>), every codeword active
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/f64abl; rm -rf $O; mkdir -p $O
timeout -k 10 120 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/cur.jsonl 2>> $O/err.log
for d in ldpc_sparc_amd/_lib_v_d*; do
  n=${d#ldpc_sparc_amd/_lib_v_}
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/$n.jsonl 2>> $O/err.log
  echo "$n"
done
timeout -k 10 120 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/cur.jsonl 2>> $O/err.log
echo done
