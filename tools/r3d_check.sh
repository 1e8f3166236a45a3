#!/bin/bash
# C4 on the two-class engine at P = 2^13: AMP parity tests, then a same-box
# A/B of the block lines (library at the previous commit in
# ldpc_sparc_amd/_lib_alt against the working build), and the single-class
# engine of the working build (SG_AMP_BLOCK=single, through the C4 probe).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3d; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_amp_gpu.py -x -q --timeout 200 --timeout-method thread -k "c4 or notebook or block" > $O/tests.log 2>&1
for i in 1 2; do
  LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_alt/libldpc_sparc_amd.so timeout -k 10 200 python bench.py --no-bp --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 2 > $O/old$i.json 2>$O/old$i.err
  timeout -k 10 200 python bench.py --no-bp --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 2 > $O/new$i.json 2>$O/new$i.err
done
timeout -k 10 300 python -u -m pytest tests/test_amp_cw2_gpu.py tests/test_amp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_all.log 2>&1
echo done
