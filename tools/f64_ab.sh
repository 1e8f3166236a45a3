#!/bin/bash
# f64 split engine: correctness (max |dNMSE| against the staged engine), GPU tests, then per-launch
# kernel times of the current build and the _lib_v_* variants (every codeword active) and the probe
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/f64ab; rm -rf $O; mkdir -p $O
timeout -k 10 120 python tools/f64_diff.py > $O/diff.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_amp_cw2d_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 120 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/cur.jsonl 2>> $O/err.log
for d in ldpc_sparc_amd/_lib_v_*; do
  [ -d "$d" ] || continue
  n=${d#ldpc_sparc_amd/_lib_v_}
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/$n.jsonl 2>> $O/err.log
done
timeout -k 10 120 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/cur.jsonl 2>> $O/err.log
timeout -k 10 200 python tools/amp_probe.py 256 f64 >> $O/probe.log 2>&1
timeout -k 10 200 python tools/amp_probe.py 256 f64 >> $O/probe.log 2>&1
echo done
