#!/bin/bash
# Timing ablation of the regular AMP engine's stage kernels (results wrong on purpose).
for sk in 0 1 2 4 3 5 6 7; do
  echo "skip=$sk"
  SG_AMP_SKIP=$sk timeout -k 10 120 python bench.py --cpu-seconds 0 --no-bp --steps 4 --warmup 1 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print({k: round(v/ r['launches'][k],4) for k,v in r['kernel_ms'].items()})"
done
