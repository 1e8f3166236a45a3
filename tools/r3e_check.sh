#!/bin/bash
# BP: grouped kernel with each variable group's first two port slots in
# registers -- parity tests, then a same-box A/B of the C3 line (library at the
# previous commit in ldpc_sparc_amd/_lib_alt against the working build).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bp_grouped_gpu.py tests/test_bp_f32_exact_gpu.py tests/test_bp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2 3; do
  LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_alt/libldpc_sparc_amd.so timeout -k 10 200 python bench.py --no-sc --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 2 --bp-steps 20 > $O/old$i.json 2>$O/old$i.err
  timeout -k 10 200 python bench.py --no-sc --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 2 --bp-steps 20 > $O/new$i.json 2>$O/new$i.err
done
echo done
