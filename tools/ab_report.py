"""Summarise gpurun_out/ab (tools/ab.sh)."""
import csv
import glob
import os

O = "gpurun_out/ab"
for f in sorted(glob.glob(f"{O}/probe_*.log")):
    lines = [l for l in open(f).read().splitlines() if l.strip()]
    print(os.path.basename(f), "|", lines[-1] if lines else "")
rows = {}
for d in sorted(glob.glob(f"{O}/ks_*")):
    p = os.path.join(d, "run_kernel_stats.csv")
    if os.path.exists(p):
        rows[os.path.basename(d)] = {r["Name"].split("(")[0][-28:]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(p))}
names = sorted({k for v in rows.values() for k in v if "reg_" in k})
print("%-30s" % "kernel", " ".join("%12s" % k[3:] for k in rows))
for n in names:
    print("%-30s" % n, " ".join("%12.1f" % rows[k].get(n, 0) for k in rows))
