#!/bin/bash
# C5 (dense MFMA path) counters: kernel trace + stats, FETCH_SIZE and
# WRITE_SIZE passes, an MFMA pass (counters chosen from rocprofv3 -L), each
# its own run of tools/concat_probe.py; summary by tools/pmc_concat.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmcc; rm -rf $O; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python tools/concat_probe.py 2 > $O/ks.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python tools/concat_probe.py 1 > $O/f.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python tools/concat_probe.py 1 > $O/w.log 2>&1
MF=""
for c in SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE; do
  grep -q "\b$c\b" $O/counters.txt && MF="$MF $c"
done
echo "mfma pass counters:$MF" > $O/mfma_counters.txt
[ -n "$MF" ] && timeout -s KILL 200 rocprofv3 --pmc $MF --output-format csv -d $O/m -o run -- python tools/concat_probe.py 1 > $O/m.log 2>&1
echo done
