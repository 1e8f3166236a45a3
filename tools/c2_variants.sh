#!/bin/bash
# Same-box A/B of split-engine build variants (_lib_v_c2*): per-launch kernel times with every codeword
# active (tools/c2_ablate.py), the current build interleaved, two rounds; then the C2 decode probe
# (tools/amp_c2_probe.py: early stop as shipped) for each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c2v; rm -rf $O; mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python tools/c2_ablate.py 256 10 3 >> $O/cur.jsonl 2>> $O/err.log
  for d in ldpc_sparc_amd/_lib_v_c2*; do
    n=${d#ldpc_sparc_amd/_lib_v_}
    LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/c2_ablate.py 256 10 3 >> $O/$n.jsonl 2>> $O/err.log
  done
  echo "round $i"
done
for i in 1 2; do
  timeout -k 10 120 python tools/amp_c2_probe.py 256 4 >> $O/probe_cur.log 2>&1
  for d in ldpc_sparc_amd/_lib_v_c2*; do
    n=${d#ldpc_sparc_amd/_lib_v_}
    LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/amp_c2_probe.py 256 4 >> $O/probe_$n.log 2>&1
  done
done
echo done
