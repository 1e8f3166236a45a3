#!/bin/bash
# Same-box A/B of two library builds on the C2 bench line: the committed
# build (ldpc_sparc_amd/_lib) against an alternative linked by hand into
# ldpc_sparc_amd/_lib_alt (e.g. an older amp_cw.o), loaded through
# LDPC_SPARC_AMD_LIB, interleaved twice.
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/ab; mkdir -p gpurun_out/ab
for i in 1 2; do
  LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_alt/libldpc_sparc_amd.so timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 > gpurun_out/ab/old$i.json 2>/dev/null
  timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 > gpurun_out/ab/new$i.json 2>/dev/null
done
