#!/bin/bash
# Same-box A/B of the C3 bench line under environment settings, interleaved
# twice: bash tools/ab_env_bp.sh "name:VAR=val VAR2=val" "name2:..." ...
# (an empty setting after the colon runs the defaults).  Optionally first
# runs the BP GPU tests when AB_TESTS=1.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abenv; rm -rf $O; mkdir -p $O
if [ "${AB_TESTS:-0}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bp_grouped_gpu.py tests/test_bp_f32_exact_gpu.py tests/test_bp_gpu.py > $O/tests.log 2>&1
fi
A="--no-sc --no-sc-notebook --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 1 --warmup 1 --bp-steps 10 --bp-ebn0-extra"
for i in 1 2; do
  for cfg in "$@"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 200 python bench.py $A > $O/$name.$i.json 2> $O/$name.$i.err
  done
done
python - "$@" <<'PY'
import json, sys
for cfg in sys.argv[1:]:
    name = cfg.split(":")[0]
    for i in (1, 2):
        d = json.loads(open(f"gpurun_out/abenv/{name}.{i}.json").read().strip().splitlines()[-1])
        bp = d["bp"]
        print(f"{name:12s} {i} {bp['value']:.4g} cw/s  frac {bp['roofline']['frac']:.4f}  {bp['roofline']['kernel']}")
PY
