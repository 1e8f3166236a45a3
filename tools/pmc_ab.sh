#!/bin/bash
# HBM (fabric) traffic of the C2 kernels for the current build ("base") and every
# ldpc_sparc_amd/_lib_v_<name>/: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in
# separate passes over a short C2-only bench run each, summarised by
# tools/pmc_ab.py (bytes per codeword-iteration per kernel, FETCH x2 on gfx950).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmcab; rm -rf $O; mkdir -p $O
A="--no-bp --no-sc --no-sc-notebook --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 2 --warmup 1"
run() {  # name libpath
  for c in FETCH_SIZE WRITE_SIZE; do
    LDPC_SPARC_AMD_LIB=$2 timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $O/$1_$c -o run -- python bench.py $A --detail-dir $O/d_$1 > $O/$1_$c.json 2> $O/$1_$c.err
  done
}
run base $PWD/ldpc_sparc_amd/_lib/libldpc_sparc_amd.so
for d in ldpc_sparc_amd/_lib_v_*; do
  [ -d "$d" ] || continue
  run ${d#ldpc_sparc_amd/_lib_v_} $PWD/$d/libldpc_sparc_amd.so
done
python tools/pmc_ab.py $O > $O/summary.txt 2>&1
