#!/bin/bash
# One _lib_v_<name> variant of the f64 split engine against the current build: NMSE agreement with the
# staged engine and the f64 GPU tests under the variant, then per-launch kernel times (every codeword
# active) and the decode probe of both, interleaved:  tools/f64_variant_check.sh <name>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=$PWD/ldpc_sparc_amd/_lib_v_$1/libldpc_sparc_amd.so
O=gpurun_out/f64v_$1; rm -rf $O; mkdir -p $O
LDPC_SPARC_AMD_LIB=$V timeout -k 10 120 python tools/f64_diff.py > $O/diff.log 2>&1
LDPC_SPARC_AMD_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_amp_cw2d_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/cur.jsonl 2>> $O/err.log
  LDPC_SPARC_AMD_LIB=$V timeout -k 10 120 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/var.jsonl 2>> $O/err.log
done
for i in 1 2; do
  timeout -k 10 200 python tools/amp_probe.py 256 f64 >> $O/probe_cur.log 2>&1
  LDPC_SPARC_AMD_LIB=$V timeout -k 10 200 python tools/amp_probe.py 256 f64 >> $O/probe_var.log 2>&1
done
echo done
