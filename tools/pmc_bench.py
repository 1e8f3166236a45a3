"""Per-kernel HBM traffic of a bench run from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), corrected as MI355X_MICROARCH.md "HBM" prescribes:
FETCH_SIZE (KB) x2 on gfx950 (wide coalesced reads tally half), WRITE_SIZE
(KB) as is.  Bytes per dispatch, and per unit of work for the kernels whose
unit the bench line states (C3 codeword-iterations, C4 codeword-iterations).

usage: python tools/pmc_bench.py FETCH.csv WRITE.csv bench.json out.json
(C5: the gemm_f32_mfma dispatches give the "concat" section's bytes per launch;
tools/pmc_concat.sh adds its MFMA-busy fraction)"""
import collections
import csv
import hashlib
import json
import os
import sys

LIB = os.environ.get("LDPC_SPARC_AMD_LIB") or os.path.join(  # the library the profiled run loaded
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ldpc_sparc_amd", "_lib", "libldpc_sparc_amd.so")


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
if bench.get("detail") and os.path.exists(bench["detail"]):  # the compact line names the full record
    bench = json.load(open(bench["detail"]))
per = {}
for k in sorted(set(fetch) | set(write)):
    d = max(nd.get(k, 1), 1)
    per[k] = {"dispatches": d, "read_bytes_per_dispatch": 2.0 * fetch.get(k, 0.0) * 1024 / d,
              "write_bytes_per_dispatch": write.get(k, 0.0) * 1024 / d}
out = {"kernels": per, "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; FETCH x2 (gfx950)",
       "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16]}  # the build these bytes belong to
rf = bench.get("roofline", {})
c2k = [n for n in per if n.startswith("cw2_")]
cwk = next((n for n in per if n.startswith("cw_iter")), None)
if c2k and rf.get("codeword_iterations_per_launch"):
    # split engine: every cw2_* dispatch of the decodes over the codeword-iterations they ran
    # (cw2_az runs once per iteration of the batch)
    tot = sum((per[k]["read_bytes_per_dispatch"] + per[k]["write_bytes_per_dispatch"]) * per[k]["dispatches"]
              for k in c2k)
    naz = sum(per[k]["dispatches"] for k in c2k if k.startswith("cw2_az"))
    cwit = rf["codeword_iterations_per_launch"] * naz
    out["amp"] = {"kernel": "+".join(sorted(c2k)), "hbm_bytes_per_iteration_launch_group": tot / max(naz, 1),
                  "hbm_bytes_per_codeword_iteration": tot / cwit,
                  "codeword_iterations_per_launch": rf["codeword_iterations_per_launch"],
                  "per_kernel_bytes_per_codeword_iteration": {
                      k: (per[k]["read_bytes_per_dispatch"] + per[k]["write_bytes_per_dispatch"]) * per[k][
                          "dispatches"] / cwit for k in c2k},
                  "algorithmic_bytes_per_codeword_iteration": bench.get("roofline_hbm", {}).get(
                      "algorithmic_bytes_per_codeword_iteration")}
elif cwk and rf.get("codeword_iterations_per_launch"):
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
    kn = str(bp["roofline"].get("kernel") or "bp_flood_kernel<float,2,8,").replace(" ", "")
    k = next((n for n in per if n.replace(" ", "").startswith(kn)), None)
    if k:
        b = per[k]["read_bytes_per_dispatch"] + per[k]["write_bytes_per_dispatch"]
        out["bp"] = {"kernel": k, "hbm_bytes_per_codeword_iteration": b / units,
                     "algorithmic_bytes_per_codeword_iteration": bp.get("roofline_hbm", bp["roofline"]).get(
                         "algorithmic_bytes_per_codeword_iteration"),
                     "codeword_iterations_per_dispatch": units}
def windows(path, counter, engine_prefix):
    """HBM bytes of every dispatch between the first and the last dispatch
    of an engine's kernels (its decodes, with their control kernels and
    memsets), and the number of that engine's az dispatches in it."""
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
            rows.append((int(r["Dispatch_Id"]), name, float(r["Counter_Value"])))
    ab, az = engine_prefix
    ids = [i for i, n, _ in rows if n.startswith(ab + az)]
    if not ids:
        return 0.0, 0
    lo, hi = min(ids), max(ids)
    tot = sum(v for i, _, v in rows if lo <= i <= hi)
    naz = len({i for i, n, _ in rows if n.startswith(az)})
    return tot, naz


# (Ab, Az) kernel-name prefixes of each line's engine: C4 runs the two-class engine at P = 2^13
# (blk2_*<13, M/64>; the single-class blk_* under SG_AMP_BLOCK=single), the notebook at P = 2^14
for key, prefix in (("sc", (("blk_ab", "blk2_ab<13"), ("blk_az", "blk2_az<13"))),
                    ("sc_notebook", (("blk2_ab<14",), ("blk2_az<14",)))):
    line = bench.get(key)
    if not line or not line.get("roofline", {}).get("launches"):
        continue
    fb, naz = windows(sys.argv[1], "FETCH_SIZE", prefix)
    wb, _ = windows(sys.argv[2], "WRITE_SIZE", prefix)
    steps_t = max(1, round(line["roofline"]["launches"].get("az_passB", 0) / max(1, line["avg_iterations"])))
    az_per_decode = line["roofline"]["launches"].get("az_passB", 0) / max(1, steps_t)
    decodes = naz / az_per_decode if az_per_decode else 0
    units = decodes * line["batch_per_gpu"] * line["avg_iterations"]
    b = 2.0 * fb * 1024 + wb * 1024
    out[key] = {"engine_kernels": "|".join(prefix[0] + prefix[1]), "decodes_in_window": decodes,
                "codeword_iterations": units,
                "hbm_bytes_per_codeword_iteration": b / units if units else None,
                "note": "FETCH x2 + WRITE of every dispatch from the first to the last block-engine dispatch "
                        "(decodes incl. control kernels), over the executed codeword-iterations"}

json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out, indent=1))
