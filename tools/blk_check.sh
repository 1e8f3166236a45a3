#!/bin/bash
# Block engines (C4 and the notebook geometry) after an FFT change: their GPU
# tests and the general-path AMP tests that share fft.hpp, then the sc and
# sc_notebook bench lines, current build against the base variant.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/blk; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_amp_gpu.py > $O/tests.log 2>&1
A="--no-bp --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 1 --warmup 1 --bp-ebn0-extra --sc-steps 2"
timeout -k 10 300 python bench.py $A > $O/cur.json 2> $O/cur.err
LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_v_base/libldpc_sparc_amd.so timeout -k 10 300 python bench.py $A > $O/base.json 2> $O/base.err
python - <<'PY'
import json
for f in ("cur", "base"):
    d = json.loads(open(f"gpurun_out/blk/{f}.json").read().strip().splitlines()[-1])
    print(f, "C2", round(d["value"]), "sc", round(d["sc"]["value"]), d["sc"]["roofline"]["frac"],
          "nb", round(d["sc_notebook"]["value"]), d["sc_notebook"]["roofline"]["frac"])
PY
