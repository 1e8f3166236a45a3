#!/bin/bash
# C4 (L = 1024) on the single-class block engine (default: one 1024-thread workgroup per CU) against the two-class
# form (SG_AMP_BLOCK=two-class: two 512-thread workgroups per CU) with the split engine's phase priority
# (_lib_v_b2p: -DB2_PRIO_REST=1) and without it: codewords/s by tools/amp_c4_probe.py (three rounds), then SQ
# counters (two passes of 8) of each form over one probe run.  Output gpurun_out/c4ab/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4ab; rm -rf $O; mkdir -p $O
P=$PWD/ldpc_sparc_amd/_lib_v_b2p/libldpc_sparc_amd.so
for i in 1 2 3; do
  timeout -k 10 120 python tools/amp_c4_probe.py 256 3 1.5 1024 >> $O/single.txt 2>&1
  SG_AMP_BLOCK=two-class timeout -k 10 120 python tools/amp_c4_probe.py 256 3 1.5 1024 >> $O/two.txt 2>&1
  SG_AMP_BLOCK=two-class LDPC_SPARC_AMD_LIB=$P timeout -k 10 120 python tools/amp_c4_probe.py 256 3 1.5 1024 >> $O/two_prio.txt 2>&1
done
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
C2="SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
sq() {  # name env...
  local n=$1; shift
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $O/$n/p1 -o run -- python tools/amp_c4_probe.py 256 1 1.5 1024 > $O/$n.p1.log 2>&1
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $O/$n/p2 -o run -- python tools/amp_c4_probe.py 256 1 1.5 1024 > $O/$n.p2.log 2>&1
  python tools/pmc_sq_bench.py $O/$n/p1/run_counter_collection.csv $O/$n/p2/run_counter_collection.csv $O/$n/sq.json blk > $O/$n.sq.log 2>&1
}
sq single X=1
sq two SG_AMP_BLOCK=two-class
sq two_prio SG_AMP_BLOCK=two-class LDPC_SPARC_AMD_LIB=$P
echo done
