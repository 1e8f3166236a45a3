#!/bin/bash
# Phase stamps and C2 probe of every saved library variant (_lib_v_*) beside
# the current build (diagnostic A/B; variants may be timing-only builds).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cvt; rm -rf $O; mkdir -p $O
timeout -k 10 120 python tools/cw2_tprof.py > $O/tprof_cur.log 2>&1
timeout -k 10 120 python tools/amp_c2_probe.py 256 4 > $O/probe_cur.log 2>&1
for d in ldpc_sparc_amd/_lib_v_*; do
  [ -d "$d" ] || continue
  n=${d#ldpc_sparc_amd/_lib_v_}
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/cw2_tprof.py > $O/tprof_$n.log 2>&1
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/amp_c2_probe.py 256 4 > $O/probe_$n.log 2>&1
done
echo done
