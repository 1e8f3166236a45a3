#!/bin/bash
# Locality what-if: skip=32 makes the stage-1 kernels load s / U rows of codeword cw & 7 (cache resident).
cd "$GRAFT_REPO_ROOT"
for sk in 64 32; do
  echo "skip=$sk"
  SG_AMP_SKIP=$sk timeout -k 10 120 python bench.py --cpu-seconds 0 --no-bp --no-concat --steps 4 --warmup 1 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print({k: round(v/ r['launches'][k],4) for k,v in r['kernel_ms'].items()})"
done
