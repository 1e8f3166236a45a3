#!/bin/bash
# Split engine quick loop: parity tests, phase stamps, C2 probe A/B against
# the one-workgroup engine (same box).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cw2q; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_amp_cw2_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 120 python tools/cw2_tprof.py > $O/tprof.log 2>&1
timeout -k 10 120 python tools/amp_c2_probe.py 256 5 > $O/probe_cw2.log 2>&1
timeout -k 10 120 env SG_AMP_CW2=0 python tools/amp_c2_probe.py 256 5 > $O/probe_cw1.log 2>&1
for d in ldpc_sparc_amd/_lib_v_*; do
  [ -d "$d" ] || continue
  n=${d#ldpc_sparc_amd/_lib_v_}
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/amp_c2_probe.py 256 5 > $O/probe_v_$n.log 2>&1
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/cw2_tprof.py > $O/tprof_v_$n.log 2>&1
done
echo done
