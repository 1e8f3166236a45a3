#!/bin/bash
# Same-box A/B of two library builds on the C4 (spatially coupled, block
# engine) bench line: the alternative in ldpc_sparc_amd/_lib_alt (loaded
# through LDPC_SPARC_AMD_LIB) against the current build, interleaved twice.
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/absc; mkdir -p gpurun_out/absc
A="--no-bp --no-concat --no-r13 --cpu-seconds 0 --steps 1 --warmup 1 --sc-steps 3"
for i in 1 2; do
  LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_alt/libldpc_sparc_amd.so timeout -k 10 200 python bench.py $A > gpurun_out/absc/old$i.json 2>/dev/null
  timeout -k 10 200 python bench.py $A > gpurun_out/absc/new$i.json 2>/dev/null
done
