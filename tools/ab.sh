#!/bin/bash
# A/B timing of two builds of the library (abtest/base.so, abtest/new.so):
# C2 probe and rocprofv3 kernel stats, interleaved.  Report: tools/ab_report.py
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
for round in 1 2; do
  for v in base new; do
    LDPC_SPARC_AMD_LIB=$PWD/abtest/$v.so timeout -k 10 300 python tools/amp_c2_probe.py 256 3 1.5 > $O/probe_${v}_$round.log 2>&1
    LDPC_SPARC_AMD_LIB=$PWD/abtest/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_${v}_$round -o run -- python tools/amp_c2_probe.py 256 2 1.5 > $O/prof_${v}_$round.log 2>&1
  done
done
