#!/bin/bash
# Finer ablation of the stage-1 kernels: 8 = no section reduction, 16 = no LDS zeroing.
for sk in 0 7 15 23 31 8 16; do
  echo "skip=$sk"
  SG_AMP_SKIP=$sk timeout -k 10 120 python bench.py --cpu-seconds 0 --no-bp --no-concat --steps 4 --warmup 1 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print({k: round(v/ r['launches'][k],4) for k,v in r['kernel_ms'].items()})"
done
