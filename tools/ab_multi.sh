#!/bin/bash
# Same-box A/B of several library builds on the C2 bench line: the current
# build ("base") and every ldpc_sparc_amd/_lib_v_<name>/ (loaded through
# LDPC_SPARC_AMD_LIB), interleaved AB_ROUNDS times (default 2).  Output:
# gpurun_out/abm/<name><i>.json (the line) and gpurun_out/abm/d_<name><i>/ (the
# detail record).  AB_ARGS overrides the bench arguments (default: the C2 line only).
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/abm; mkdir -p gpurun_out/abm
A=${AB_ARGS:-"--no-bp --no-sc --no-sc-notebook --no-concat --no-r13 --no-f64 --cpu-seconds 0"}
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  timeout -k 10 200 python bench.py $A --detail-dir gpurun_out/abm/d_base$i > gpurun_out/abm/base$i.json 2>/dev/null
  for d in ldpc_sparc_amd/_lib_v_*; do
    n=${d#ldpc_sparc_amd/_lib_v_}
    LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 200 python bench.py $A --detail-dir gpurun_out/abm/d_$n$i > gpurun_out/abm/$n$i.json 2>/dev/null
  done
done
python tools/ab_summary.py gpurun_out/abm > gpurun_out/abm/summary.txt
