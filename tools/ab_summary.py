"""Prints value / roofline frac of every line in gpurun_out/ab_*/{old,new}N.json."""
import glob
import json
import os
import sys


def lines(d):
    out = {}
    for k in ("", "amp_r13", "amp_f64", "bp", "sc", "sc_notebook", "concat"):
        o = d if k == "" else d.get(k)
        if isinstance(o, dict) and "value" in o:
            rf = o.get("roofline") or {}
            out[k or "c2"] = (o["value"], rf.get("frac"))
    return out


for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    try:
        d = json.loads([l for l in open(f).read().splitlines() if l.startswith("{")][-1])
    except (IndexError, ValueError):
        print(os.path.basename(f), "no line")
        continue
    print(os.path.basename(f), " ".join(f"{k}={v:.6g}" + (f"({fr:.4f})" if fr else "") for k, (v, fr) in
                                        lines(d).items()))
