#!/bin/bash
# C2 throughput of both AMP engines over the batch size (engine-choice check).
set -e
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/bsw; mkdir -p gpurun_out/bsw
for B in 128 256 384 512; do
  for E in cw staged; do
    SG_AMP_ENGINE=$E timeout -k 10 200 python bench.py --no-bp --no-sc --no-concat --no-r13 --cpu-seconds 0 --batch $B --steps 5 > gpurun_out/bsw/${E}_${B}.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/bsw/${E}_${B}.json'));print('$E',$B,round(d['value']),d['roofline']['engine'])" >> gpurun_out/bsw/summary.txt
  done
done
