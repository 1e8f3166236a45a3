#!/bin/bash
# Stage-1 kernel ablation (results wrong on purpose): 1 FFT, 2 gather/scatter,
# 4 row I/O, 8 section reduction, 16 LDS zeroing; ms per launch.
cd "$GRAFT_REPO_ROOT"
for sk in 0 1 2 4 8 16 31; do
  echo "skip=$sk"
  SG_AMP_SKIP=$sk timeout -k 10 120 python bench.py --cpu-seconds 0 --no-bp --no-concat --steps 4 --warmup 1 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print({k: round(v/ r['launches'][k],4) for k,v in r['kernel_ms'].items()})"
done
