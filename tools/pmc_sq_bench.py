"""Per-kernel SQ counter summary of tools/pmc_sq_bench.sh's two passes:
waits, VALU and LDS issue as fractions of wave cycles, LDS bank-conflict
cycles as a fraction of LDS-array cycles (SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE, MI355X_MICROARCH.md LDS section).

With the bench line of the profiled run (bench.json), an "amp" section
gives the split engine's VALU wave-instructions per codeword-iteration (all
cw2_* kernels over the codeword-iterations they ran); bench.py turns it into
roofline.valu_issue_frac and roofline.flops_per_lane_instr.  "lib_sha256"
names the library build the counters belong to (bench.py uses a file only
for that build).

usage: python tools/pmc_sq_bench.py pass1.csv pass2.csv out.json [bench.json] [kernel-prefix ...]"""
import hashlib
import os
import collections
import csv
import json
import sys


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        n[name].add(r["Dispatch_Id"])
    return agg, n


a1, n1 = load(sys.argv[1])
a2, _ = load(sys.argv[2])
bench_json = sys.argv[4] if len(sys.argv) > 4 and sys.argv[4].endswith(".json") else None
out = {}
for k in sorted(a1):
    prefixes = sys.argv[5 if bench_json else 4:] or ["cw_iter", "cw2_", "cw2d_", "bp_flood_kernel", "bp_grouped",
                                                      "blk", "gemm_", "dense_", "control_kernel"]
    if not any(k.startswith(pf) for pf in prefixes):
        continue
    c = dict(a1[k])
    c.update(a2.get(k, {}))
    wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    lds = c.get("SQ_LDS_IDX_ACTIVE", 0.0) or 1.0
    out[k] = {"dispatches": len(n1[k]), "counters": c,
              "wait_any_frac": c.get("SQ_WAIT_ANY", 0) / wc,
              "active_any_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
              "valu_active_frac": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
              "lds_active_frac": c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
              "wait_inst_lds_frac": c.get("SQ_WAIT_INST_LDS", 0) / wc,
              "lds_bank_conflict_frac": c.get("SQ_LDS_BANK_CONFLICT", 0) / lds,
              "lds_insts_per_wave": c.get("SQ_INSTS_LDS", 0) / max(c.get("SQ_WAVES", 1), 1),
              "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1)}
LIB = os.environ.get("LDPC_SPARC_AMD_LIB") or os.path.join(  # the library the profiled run loaded
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ldpc_sparc_amd", "_lib", "libldpc_sparc_amd.so")
res = {"kernels": out, "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16],
       "method": "rocprofv3 --pmc, two passes of 8 SQ counters over a short bench.py run (tools/pmc_sq_bench.sh: "
                 + os.environ.get("SQ_ARGS_USED", "") + "); fractions of SQ_WAVE_CYCLES (summed over waves)"}
if bench_json:
    lines = [l for l in open(bench_json).read().splitlines() if l.startswith("{")]
    rf = json.loads(lines[-1]).get("roofline", {}) if lines else {}
    c2k = [k for k in out if k.startswith("cw2_") and not k.startswith("cw2d_")]
    naz = sum(out[k]["dispatches"] for k in c2k if k.startswith("cw2_az"))
    if c2k and naz and rf.get("codeword_iterations_per_launch"):
        cwit = rf["codeword_iterations_per_launch"] * naz
        tot = lambda c: sum(out[k]["counters"].get(c, 0.0) for k in c2k)  # noqa: E731
        res["amp"] = {"kernels": sorted(c2k), "codeword_iterations": cwit,
                      "valu_wave_insts_per_codeword_iteration": tot("SQ_INSTS_VALU") / cwit,
                      "lds_wave_insts_per_codeword_iteration": tot("SQ_INSTS_LDS") / cwit,
                      "salu_wave_insts_per_codeword_iteration": tot("SQ_INSTS_SALU") / cwit,
                      "wait_any_frac": tot("SQ_WAIT_ANY") / max(tot("SQ_WAVE_CYCLES"), 1.0),
                      "lds_bank_conflict_frac": tot("SQ_LDS_BANK_CONFLICT") / max(tot("SQ_LDS_IDX_ACTIVE"), 1.0)}
json.dump(res, open(sys.argv[3], "w"), indent=1)
print(json.dumps({k: {kk: v for kk, v in d.items() if kk != "counters"} for k, d in out.items()}, indent=1))
