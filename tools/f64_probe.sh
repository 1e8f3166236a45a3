#!/bin/bash
# f64 C2: the split engine (amp_cw2d.hip) against the staged engine, per-launch kernel times with every
# codeword active (tools/c2_ablate.py ... f64) and the decode probe (tools/amp_probe.py 256 f64)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/f64; mkdir -p $O
timeout -k 10 200 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/abl_cw.jsonl 2>> $O/err.log
SG_AMP_ENGINE=staged timeout -k 10 200 python tools/c2_ablate.py 256 10 2 1.5 f64 >> $O/abl_staged.jsonl 2>> $O/err.log
for i in 1 2; do
  timeout -k 10 200 python tools/amp_probe.py 256 f64 >> $O/probe_auto.log 2>&1
  SG_AMP_ENGINE=staged timeout -k 10 200 python tools/amp_probe.py 256 f64 >> $O/probe_staged.log 2>&1
done
echo done
