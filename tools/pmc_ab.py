"""Summary of tools/pmc_ab.sh: per build, the C2 kernels' fabric bytes per
codeword-iteration (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM
section), from the bench line's codeword-iterations per launch."""
import collections
import csv
import glob
import json
import os
import sys


def load(path, counter):
    agg, n = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
        agg[name] += float(r["Counter_Value"])
        n[name].add(r["Dispatch_Id"])
    return agg, {k: len(v) for k, v in n.items()}


O = sys.argv[1]
for fj in sorted(glob.glob(os.path.join(O, "*_FETCH_SIZE.json"))):
    name = os.path.basename(fj)[:-len("_FETCH_SIZE.json")]
    fc = glob.glob(os.path.join(O, f"{name}_FETCH_SIZE", "run_counter_collection.csv"))
    wc = glob.glob(os.path.join(O, f"{name}_WRITE_SIZE", "run_counter_collection.csv"))
    if not fc or not wc:
        print(name, "missing counters")
        continue
    f, nd = load(fc[0], "FETCH_SIZE")
    w, _ = load(wc[0], "WRITE_SIZE")
    line = json.loads([l for l in open(fj).read().splitlines() if l.startswith("{")][-1])
    cpl = line["roofline"]["codeword_iterations_per_launch"]
    naz = sum(v for k, v in nd.items() if k.startswith("cw2_az"))
    cwit = cpl * naz
    per = {k: (2 * f.get(k, 0) + w.get(k, 0)) * 1024 / cwit for k in f if k.startswith("cw2_")}
    print(f"{name}: total {sum(per.values()) / 1e6:.3f} MB per codeword-iteration; " +
          ", ".join(f"{k} {v / 1e6:.3f}" for k, v in sorted(per.items())))
