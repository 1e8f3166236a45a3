#!/bin/bash
# BP grouped min-sum kernel: GPU parity tests, then a same-box A/B of the C3
# bench line against the table kernel (SG_BP_GROUPED=0), interleaved twice.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abgrp; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bp_grouped_gpu.py tests/test_bp_f32_exact_gpu.py tests/test_bp_gpu.py > $O/tests.log 2>&1
A="--no-sc --no-sc-notebook --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 1 --warmup 1 --bp-steps 10 --bp-ebn0-extra 1.0 1.5"
for i in 1 2; do
  SG_BP_GROUPED=0 timeout -k 10 200 python bench.py $A > $O/old$i.json 2>$O/old$i.err
  timeout -k 10 200 python bench.py $A > $O/new$i.json 2>$O/new$i.err
done
python - <<'PY'
import json
for f in ["old1", "new1", "old2", "new2"]:
    d = json.loads(open(f"gpurun_out/abgrp/{f}.json").read().strip().splitlines()[-1])
    bp = d.get("bp", d)
    print(f, json.dumps({k: bp.get(k) for k in ("value", "ms_per_step", "roofline")})[:400])
    for e in d.get("bp_ebn0", []) or []:
        print("   ", json.dumps(e)[:300])
PY
