"""Summarise gpurun_out/quick (tools/quick.sh)."""
import collections
import csv
import glob
import os

O = "gpurun_out/quick"
for f in sorted(glob.glob(f"{O}/*.log")):
    if "prof" in f or "pmc" in f:
        continue
    lines = [l for l in open(f).read().splitlines() if l.strip()]
    print(os.path.basename(f), "|", lines[-1] if lines else "")
p = f"{O}/ks/run_kernel_stats.csv"
if os.path.exists(p):
    for r in list(csv.DictReader(open(p)))[:8]:
        print("  %-45s %4s %9.1f us" % (r["Name"][:45], r["Calls"], float(r["AverageNs"]) / 1e3))
p = f"{O}/pmc/run_counter_collection.csv"
if os.path.exists(p):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            n[k] += 1
    for k, d in agg.items():
        if "reg_a" not in k and "reg_m" not in k:
            continue
        w = d["SQ_WAVES"]
        print("  %-40s VALU/wave %6.0f LDS/wave %5.0f confl %.2f waitany %.2f valu-active %.2f" % (
            k, d["SQ_INSTS_VALU"] / w, d["SQ_INSTS_LDS"] / w, d["SQ_LDS_BANK_CONFLICT"] / max(1, d["SQ_LDS_IDX_ACTIVE"]),
            d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], d["SQ_ACTIVE_INST_VALU"] / d["SQ_WAVE_CYCLES"]))
