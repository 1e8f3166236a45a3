"""Summarise gpurun_out/check (tools/amp_check.sh)."""
import csv
import os

O = "gpurun_out/check"
for name in ("tprof.log",):
    p = os.path.join(O, name)
    if os.path.exists(p):
        print("".join(l for l in open(p) if l.strip()), end="")
for name in ("probe.log", "tests.log"):
    p = os.path.join(O, name)
    if os.path.exists(p):
        lines = [l for l in open(p).read().splitlines() if l.strip()]
        print(name, "|", lines[-1] if lines else "")
p = os.path.join(O, "ks", "run_kernel_stats.csv")
if os.path.exists(p):
    for r in list(csv.DictReader(open(p)))[:8]:
        print("  %-45s %5s %9.1f us" % (r["Name"][:45], r["Calls"], float(r["AverageNs"]) / 1e3))
p = os.path.join(O, "diag.log")
if os.path.exists(p):
    for l in open(p):
        f = l.split()
        if len(f) > 6 and f[4] != f[6]:
            print("f32 t_final differs:", f[0], "ref", f[2], "f64", f[4], "f32", f[6])
