"""Summary of tools/pmc_concat.sh: per GEMM launch (gemm_f32_glds / gemm_f32_mfma) the HBM bytes
(FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md gfx950 correction), the
average duration from the kernel-trace stats, and the MFMA counters; merged as
the "concat" section into the round's PMC traffic file (bench.py reads
concat.hbm_bytes_per_gemm_launch and concat.mfma_busy_frac from it).

MFMA-busy: SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CU_CYCLES x 4 SIMDs) over the
GEMM dispatches when both counters exist; the flop-based fraction (bench.py)
is the primary figure.

usage: python tools/pmc_concat.py DIR traffic.json"""
import collections
import csv
import glob
import json
import os
import sys

d, tfile = sys.argv[1], sys.argv[2]


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    return agg, {k: len(v) for k, v in n.items()}


gk = "gemm_f32_"  # gemm_f32_glds (LDS-DMA staging, default) or gemm_f32_mfma
f, nf = load(os.path.join(d, "f", "run_counter_collection.csv"))
w, _ = load(os.path.join(d, "w", "run_counter_collection.csv"))
fk = next(k for k in f if k.startswith(gk))
nd = nf[fk]
rb = 2.0 * f[fk]["FETCH_SIZE"] * 1024 / nd
wb = w[fk]["WRITE_SIZE"] * 1024 / nd
sec = {"kernel": fk, "dispatches_per_decode": nd, "read_bytes_per_launch": rb, "write_bytes_per_launch": wb,
       "hbm_bytes_per_gemm_launch": rb + wb}
ks = glob.glob(os.path.join(d, "ks", "*kernel_stats.csv"))
if ks:
    for r in csv.DictReader(open(ks[0])):
        if r["Name"].replace("void ", "").replace("sg::", "").startswith(gk):
            sec["avg_duration_ns"] = float(r["AverageNs"])
            sec["kernel_stats_file"] = os.path.basename(ks[0])
mp = os.path.join(d, "m", "run_counter_collection.csv")
if os.path.exists(mp):
    m, _ = load(mp)
    mk = next((k for k in m if k.startswith(gk)), None)
    if mk:
        c = dict(m[mk])
        sec["mfma_counters_per_decode"] = c
        if c.get("SQ_VALU_MFMA_BUSY_CYCLES") and c.get("SQ_BUSY_CU_CYCLES"):
            sec["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (4.0 * c["SQ_BUSY_CU_CYCLES"])
out = json.load(open(tfile)) if os.path.exists(tfile) else {}
out["concat"] = sec
json.dump(out, open(tfile, "w"), indent=1)
print(json.dumps(sec, indent=1))
