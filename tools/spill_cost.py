"""Where the register spills of each kernel sit: inside a loop or not.

Compiles every ldpc_sparc_amd/csrc/*.hip to gfx950 assembly with the
Makefile's flags (as tools/spill_check.sh does) and, for every kernel whose
metadata reports VGPR or SGPR spills, counts the spill instructions by the
loop depth of the basic block that holds them (LLVM annotates every block
inside a loop with "; in Loop: ... Depth=N" or "Loop Header ... Depth=N"):

  * SGPR spills are v_writelane_b32 / v_readlane_b32 (the library's kernels use
    no lane intrinsics other than readfirstlane, so every such instruction is
    a spill or a reload);
  * VGPR spills are scratch_store / scratch_load (or buffer_* ... offen with
    the scratch resource) instructions.

A spill instruction outside every loop executes once per wave per launch; the
report gives, per kernel, the count at depth 0 and inside loops, and with
--dispatched FILE only the kernels named in FILE (one demangled name per line,
e.g. from a rocprofv3 kernel trace).

usage: python tools/spill_cost.py [--dispatched FILE] [--json OUT]
"""
import argparse
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "ldpc_sparc_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(REPO, "include"), "--cuda-device-only",
         "-S", "-x", "hip"]
EXTRA = {"bp": ["-ffp-contract=off"], "bp_grouped": ["-ffp-contract=off", "-fno-honor-nans"]}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return dict(zip(names, out))


def compile_all(tmp):
    procs = []
    for f in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        b = os.path.basename(f)[:-4]
        out = os.path.join(tmp, b + ".s")
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc"] + FLAGS + EXTRA.get(b, []) + [f, "-o", out],
                                      stderr=subprocess.DEVNULL))
    for p in procs:
        p.wait()
    return sorted(glob.glob(os.path.join(tmp, "*.s")))


SPILL_S = re.compile(r"^\s*v_(writelane|readlane)_b32\b")
SPILL_V = re.compile(r"^\s*(scratch_store|scratch_load)|^\s*buffer_(store|load)_dword\S*\s.*\boffen\b.*s\[0:3\]")
DEPTH = re.compile(r"Depth=(\d+)")


def kernel_bodies(text):
    """{symbol: [lines of its body]} for every kernel (functions with .amdhsa_kernel)."""
    bodies = {}
    kernels = set(re.findall(r"\.amdhsa_kernel\s+(\S+)", text))
    cur = None
    for line in text.splitlines():
        m = re.match(r"^(\S+):\s*(;.*)?$", line)
        if m and m.group(1) in kernels:
            cur = m.group(1)
            bodies[cur] = []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):  # (a kernel may hold several s_endpgm)
                cur = None
                continue
            bodies[cur].append(line)
    return bodies


def meta_spills(text):
    res = {}
    if "amdhsa.kernels" not in text:
        return res
    for blk in text[text.index("amdhsa.kernels"):].split("  - .")[1:]:
        nm = re.search(r"\.name:\s+(\S+)", blk)
        vs = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk)
        ss = re.search(r"\.sgpr_spill_count:\s+(\d+)", blk)
        if nm and vs and ss:
            res[nm.group(1)] = (int(vs.group(1)), int(ss.group(1)))
    return res


def analyse(body):
    depth = 0
    counts = {}
    for line in body:
        if line.startswith(".LBB") or line.startswith("; %bb"):
            m = DEPTH.search(line)
            depth = int(m.group(1)) if m else 0
            counts[("maxdepth", 0)] = max(counts.get(("maxdepth", 0), 0), depth)
            continue
        if SPILL_S.match(line) or SPILL_V.match(line):
            kind = "sgpr" if SPILL_S.match(line) else "vgpr"
            counts[(kind, depth)] = counts.get((kind, depth), 0) + 1
    return counts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dispatched", help="file of demangled kernel names that ran (others are skipped)")
    ap.add_argument("--json")
    a = ap.parse_args()
    keep = None
    if a.dispatched:
        keep = {l.strip() for l in open(a.dispatched) if l.strip()}
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        for s in compile_all(tmp):
            text = open(s).read()
            spills = meta_spills(text)
            bodies = kernel_bodies(text)
            bad = [k for k, (v, sg) in spills.items() if v or sg]
            if not bad:
                continue
            dm = demangle(bad)
            for k in bad:
                name = dm[k]
                if keep is not None and not any(name.startswith(x) or x in name for x in keep):
                    continue
                c = analyse(bodies.get(k, []))
                maxd = c.pop(("maxdepth", 0), 0)
                in_loop = sum(n for (kind, d), n in c.items() if d > 0)
                outside = sum(n for (kind, d), n in c.items() if d == 0)
                rows.append({"file": os.path.basename(s)[:-2], "kernel": name, "vgpr_spill": spills[k][0],
                             "sgpr_spill": spills[k][1], "spill_instrs_outside_loops": outside,
                             "spill_instrs_in_loops": in_loop, "deepest_loop": maxd,
                             "by_depth": {f"{kind}@{d}": n for (kind, d), n in sorted(c.items())}})
    for r in rows:
        print(f"{r['kernel'][:60]:60s} vgpr {r['vgpr_spill']:3d} sgpr {r['sgpr_spill']:3d}  "
              f"spill instrs: {r['spill_instrs_outside_loops']:3d} outside loops, {r['spill_instrs_in_loops']:3d} "
              f"in loops {r['by_depth']} (deepest loop {r['deepest_loop']})")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
