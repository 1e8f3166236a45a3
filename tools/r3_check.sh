#!/bin/bash
# Round-3 engine check: split-engine and notebook-engine GPU tests, the C2
# probe with the current build and the saved variants (_lib_v_*), and the
# notebook (sc_notebook) bench line against the base variant.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_amp_cw2_gpu.py "tests/test_amp_gpu.py::test_notebook_block2_vs_general_engine" "tests/test_amp_gpu.py::test_notebook_block2_operators" "tests/test_amp_gpu.py::test_c4_block_engine_vs_general_engine" > $O/tests.log 2>&1
timeout -k 10 120 python tools/amp_c2_probe.py 256 5 > $O/probe_cur.log 2>&1
timeout -k 10 120 python tools/cw2_tprof.py > $O/tprof.log 2>&1
for d in ldpc_sparc_amd/_lib_v_*; do
  [ -d "$d" ] || continue
  n=${d#ldpc_sparc_amd/_lib_v_}
  LDPC_SPARC_AMD_LIB=$PWD/$d/libldpc_sparc_amd.so timeout -k 10 120 python tools/amp_c2_probe.py 256 5 > $O/probe_v_$n.log 2>&1
done
A="--no-bp --no-concat --no-r13 --no-f64 --no-sc --cpu-seconds 0 --steps 1 --warmup 1 --bp-ebn0-extra"
timeout -k 10 300 python bench.py $A > $O/nb_cur.json 2> $O/nb_cur.err
LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_v_base/libldpc_sparc_amd.so timeout -k 10 300 python bench.py $A > $O/nb_base.json 2> $O/nb_base.err
python - <<'PY'
import json
for f in ("nb_cur", "nb_base"):
    d = json.loads(open(f"gpurun_out/r3c/{f}.json").read().strip().splitlines()[-1])
    nb = d.get("sc_notebook", {})
    print(f, nb.get("value"), json.dumps(nb.get("roofline"))[:300])
PY
