#!/bin/bash
# Round-3 (second session) check: the AMP parity tests, then a same-box A/B of
# the C2 line (library at HEAD in ldpc_sparc_amd/_lib_alt against the working
# build), then a kernel trace of the new build's C2 line (launch gaps).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_amp_cw2_gpu.py tests/test_amp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_alt/libldpc_sparc_amd.so timeout -k 10 200 python bench.py --no-bp --no-concat --no-r13 --no-f64 --cpu-seconds 0 > $O/old$i.json 2>/dev/null
  timeout -k 10 200 python bench.py --no-bp --no-concat --no-r13 --no-f64 --cpu-seconds 0 > $O/new$i.json 2>/dev/null
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c2 -- python bench.py --no-bp --no-concat --no-sc --no-r13 --no-f64 --cpu-seconds 0 --steps 4 > $O/prof.json 2>/dev/null
echo done
