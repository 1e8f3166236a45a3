"""Per-kernel HBM traffic of a bench run from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), corrected as MI355X_MICROARCH.md "HBM" prescribes:
FETCH_SIZE (KB) x2 on gfx950 (wide coalesced reads tally half), WRITE_SIZE
(KB) as is.  Bytes per dispatch, and per unit of work for the kernels whose
unit the bench line states (C3 codeword-iterations, C4 codeword-iterations).

usage: python tools/pmc_bench.py FETCH.csv WRITE.csv bench.json out.json"""
import collections
import csv
import json
import sys


def load(path, counter):
    agg = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
        agg[name] += float(r["Counter_Value"])
        n[name].add(r["Dispatch_Id"])
    return agg, {k: len(v) for k, v in n.items()}


fetch, nd = load(sys.argv[1], "FETCH_SIZE")
write, _ = load(sys.argv[2], "WRITE_SIZE")
lines = [l for l in open(sys.argv[3]).read().splitlines() if l.startswith("{")]
bench = json.loads(lines[-1])
per = {}
for k in sorted(set(fetch) | set(write)):
    d = max(nd.get(k, 1), 1)
    per[k] = {"dispatches": d, "read_bytes_per_dispatch": 2.0 * fetch.get(k, 0.0) * 1024 / d,
              "write_bytes_per_dispatch": write.get(k, 0.0) * 1024 / d}
out = {"kernels": per, "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; FETCH x2 (gfx950)"}
rf = bench.get("roofline", {})
cwk = next((n for n in per if n.startswith("cw_iter")), None)
if cwk and rf.get("codeword_iterations_per_launch"):
    b = per[cwk]["read_bytes_per_dispatch"] + per[cwk]["write_bytes_per_dispatch"]
    out["amp"] = {"kernel": cwk, "hbm_bytes_per_launch": b,
                  "hbm_bytes_per_codeword_iteration": b / rf["codeword_iterations_per_launch"],
                  "codeword_iterations_per_launch": rf["codeword_iterations_per_launch"],
                  "algorithmic_bytes_per_codeword_iteration": bench.get("roofline_hbm", {}).get(
                      "algorithmic_bytes_per_codeword_iteration")}
bp = bench.get("bp")
if bp:
    units = bp["batch_per_gpu"] * bp["avg_executed_iterations"]
    # the C3 line's kernel: f32 min-sum at check degree <= 8 (bp_variants add other instances)
    k = next((n for n in per if n.replace(" ", "").startswith("bp_flood_kernel<float,2,8,")), None)
    if k:
        b = per[k]["read_bytes_per_dispatch"] + per[k]["write_bytes_per_dispatch"]
        out["bp"] = {"kernel": k, "hbm_bytes_per_codeword_iteration": b / units,
                     "algorithmic_bytes_per_codeword_iteration": bp.get("roofline_hbm", bp["roofline"]).get(
                         "algorithmic_bytes_per_codeword_iteration"),
                     "codeword_iterations_per_dispatch": units}
sc = bench.get("sc")
if sc:
    units = sc["batch_per_gpu"] * sc["avg_iterations"]
    ks = [n for n in per if n.startswith("blk_")]
    b = sum((per[n]["read_bytes_per_dispatch"] + per[n]["write_bytes_per_dispatch"]) for n in ks)
    out["sc"] = {"kernels": ks, "hbm_bytes_per_codeword_iteration_approx": b / (units / (sc["avg_iterations"] + 1) * 1.0)
                 if units else None,
                 "note": "bytes of one launch of each block-engine kernel divided by the codewords of the batch "
                         "(one launch = one AMP iteration of the batch)"}
    if units:
        out["sc"]["hbm_bytes_per_codeword_iteration_approx"] = b / sc["batch_per_gpu"]
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out, indent=1))
