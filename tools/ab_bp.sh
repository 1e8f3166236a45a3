#!/bin/bash
# Same-box A/B of two library builds on the C3 (BP) bench line: the
# alternative in ldpc_sparc_amd/_lib_alt (LDPC_SPARC_AMD_LIB) against the
# current build, interleaved twice.
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/abbp; mkdir -p gpurun_out/abbp
A="--no-sc --no-sc-notebook --no-concat --no-r13 --cpu-seconds 0 --steps 1 --warmup 1 --bp-steps 10"
for i in 1 2; do
  LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_alt/libldpc_sparc_amd.so timeout -k 10 200 python bench.py $A > gpurun_out/abbp/old$i.json 2>/dev/null
  timeout -k 10 200 python bench.py $A > gpurun_out/abbp/new$i.json 2>/dev/null
done
