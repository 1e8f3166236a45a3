#!/bin/bash
set -e
# Same-box A/B of the C2 line with and without the timed region's HIP events (bench.py --timed-prof-level 2 / 0),
# interleaved three times: gpurun_out/profab/p<level>_<i>.json (profiles/r06_timed_events_ab.txt).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/profab
A="--no-bp --no-sc --no-sc-notebook --no-concat --no-r13 --no-f64 --cpu-seconds 0 --steps 20 --warmup 3"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py $A --detail-dir gpurun_out/profab/d2_$i > gpurun_out/profab/p2_$i.json 2> gpurun_out/profab/p2_$i.err
  timeout -k 10 200 python bench.py $A --timed-prof-level 0 --detail-dir gpurun_out/profab/d0_$i > gpurun_out/profab/p0_$i.json 2> gpurun_out/profab/p0_$i.err
done
