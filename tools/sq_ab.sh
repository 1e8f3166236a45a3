#!/bin/bash
# SQ counters of the C2 kernels for the current build ("base") and every
# ldpc_sparc_amd/_lib_v_<name>/ (tools/mk_variant.sh): tools/pmc_sq_bench.sh over a
# short C2-only bench run per library, output gpurun_out/sqab/<name>/sq.json.
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/sqab; mkdir -p gpurun_out/sqab
export SQ_ARGS="--no-bp --no-sc --no-sc-notebook --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 2 --warmup 1"
SQ_OUT=gpurun_out/sqab/base bash tools/pmc_sq_bench.sh
for d in ldpc_sparc_amd/_lib_v_*; do
  [ -d "$d" ] || continue
  n=${d#ldpc_sparc_amd/_lib_v_}
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so SQ_OUT=gpurun_out/sqab/$n bash tools/pmc_sq_bench.sh
done
