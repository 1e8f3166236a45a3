#!/bin/bash
# C3 kernel A/B: tools/bp_ab.py on the current build and every _lib_v_* / _lib_alt
# library, three interleaved rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bpab; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python tools/bp_ab.py 20 >> $O/cur.jsonl 2>> $O/err.log
  for d in ldpc_sparc_amd/_lib_alt ldpc_sparc_amd/_lib_v_bp*; do
    [ -f $d/libldpc_sparc_amd.so ] || continue
    n=${d#ldpc_sparc_amd/_lib_}
    LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/bp_ab.py 20 >> $O/$n.jsonl 2>> $O/err.log
  done
  echo "round $i"
done
echo done
