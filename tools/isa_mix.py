"""Static instruction mix of a kernel in a hipcc -S listing (gfx950).

usage: python tools/isa_mix.py listing.s <kernel-substring> [--loops]

Counts the instructions between the kernel's label and its .Lfunc_end by
class (VALU packed / transcendental / other, SALU, LDS, VMEM, waitcnt, nop,
barrier); with --loops, also per basic-block loop body (a block ending in a
backward branch to a label at or before it)."""
import re
import sys
from collections import Counter

TRANS = ("v_exp_f32", "v_log_f32", "v_sin_f32", "v_cos_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_rcp_iflag")


def klass(op):
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith(TRANS):
        return "valu_trans"
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def kernel_lines(path, sub):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        l = l.split(";")[0].rstrip()
        if l.endswith(":") and sub in l and not l.startswith((".", "\t")) and start is None:
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit(f"kernel {sub} not found")


def main():
    path, sub = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, sub)
    print(body[0])
    total = Counter()
    blocks, cur, label = [], Counter(), None
    labels = {}
    for l in body[1:]:
        s = l.split(";")[0].strip()
        if not s or s.startswith((";", ".")) and not s.startswith(".LBB"):
            continue
        if s.endswith(":"):
            blocks.append((label, cur))
            label, cur = s[:-1], Counter()
            labels[label] = len(blocks)
            continue
        op = s.split()[0]
        c = klass(op)
        total[c] += 1
        cur[c] += 1
        cur["_n"] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= len(blocks):
                cur["_back_to_" + tgt] = 1
    blocks.append((label, cur))
    print("total:", dict(sorted(total.items())))
    if "--loops" in sys.argv:  # every backward branch: the blocks from its target to it, summed
        for i, (lab, c) in enumerate(blocks):
            for k in c:
                if k.startswith("_back_to_"):
                    j = labels[k[len("_back_to_"):]]
                    reg = Counter()
                    for _, cc in blocks[j:i + 1]:
                        reg.update({q: v for q, v in cc.items() if not q.startswith("_b")})
                    print(f"loop {blocks[j][0]} .. {lab} ({i - j + 1} blocks):",
                          dict(sorted(reg.items())))


if __name__ == "__main__":
    main()
