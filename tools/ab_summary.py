"""Prints value / roofline frac of every bench line in <dir>/*.json (the C2
line and its companions) and, from the detail record next to it
(<dir>/d_<name>/bench_detail_*.json), the C2 kernels' times of the last
warmup step."""
import glob
import json
import os
import sys


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        try:
            line = json.loads([l for l in open(f).read().splitlines() if l.startswith("{")][-1])
        except (IndexError, ValueError):
            print(os.path.basename(f), "no line")
            continue
        rf = line.get("roofline") or {}
        parts = [f"c2={line['value']:.6g}({rf.get('frac')})"]
        for k, v in (line.get("companions") or {}).items():
            parts.append(f"{k}={v.get('value')}({v.get('frac')})")
        det = glob.glob(os.path.join(d, "d_" + os.path.basename(f)[:-5], "bench_detail_*.json"))
        if det:
            full = json.load(open(det[0]))
            km = (full.get("roofline") or {}).get("kernel_ms_last_warmup_step") or {}
            ln = (full.get("roofline") or {}).get("launches_last_warmup_step") or {}
            parts.append(" ".join(f"{k}:{v / max(ln.get(k, 1), 1):.4f}" for k, v in sorted(km.items())))
        print(os.path.basename(f), " ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
