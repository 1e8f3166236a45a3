"""Bank-conflict cost of the C3 kernel's variable pass on the host's degree-grouped layout
(capi_ldpc.cpp grp_layout through sg_ldpc_grouped_layout, no GPU), and how far the layout's
placement freedom can lower it by greedy swaps.

Cost model (as round 5's): per variable group, per port k, per 32-lane half, the largest number of
distinct message slots on one LDS bank (ds_read_b32: 2 x 32 lane groups, bank = (addr / 4) mod 32);
conflict-free = 2 cycles per group and port.  Two searches, each accepting swaps that do not raise
the cost: (var) two variables of one degree swap lanes (any groups: a variable's arithmetic does not
depend on its lane); (chk) two checks of one degree swap positions (check group, lane): the check
pass reads a check's ports at addr + 256 k + 4 lane, conflict-free for any placement, while every
variable reading one of their ports sees a new bank.

usage: python tools/bp_bank_search.py [var|chk] [std rate z] [iterations]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_bp_grouped_layout import PAIR, W, layout  # noqa: E402
from ldpc_sparc_amd.ldpc import code  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "chk"
std, rate, z = (sys.argv[2], sys.argv[3], int(sys.argv[4])) if len(sys.argv) > 4 else ("802.11n", "1/2", 81)
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 200000
c = code(std, rate, z)
lay = layout(c.vdeg, c.cdeg, c.intrlv)
vt, vd, vtab, vmap = lay["vt"], lay["vdeg"] & (PAIR - 1), lay["vtab"].astype(np.int64), lay["vmap"]
cd, ca, cv = lay["cdeg"], lay["caddr"], lay["cval"]
cgroups = [(w, q) for w in range(W) for q in range(lay["cj"]) if cd[w, q] >= 2]
gi = {g: i for i, g in enumerate(cgroups)}
addr = [int(ca[g]) for g in cgroups]
deg = [int(cd[g]) for g in cgroups]
groups = [(w, j) for w in range(W) for j in range(lay["vj"]) if vd[w, j] > 0]


def decode(s):  # message slot -> (check group index, lane, port)
    for i, (a, d) in enumerate(zip(addr, deg)):
        if a <= s < a + 256 * d:
            return i, ((s - a) % 256) // 4, (s - a) // 256
    raise ValueError(s)


# every read of the variable pass as (check id = (group, lane) of the initial layout, port), None = padding lane
R = {g: [[None if vmap[g][l] < 0 else decode(int(vtab[vt[g] + 64 * k + l])) for l in range(64)]
         for k in range(vd[g])] for g in groups}
place = {(i, l): (i, l) for i in range(len(cgroups)) for l in range(64)}


def slot(e):
    i, l = place[(e[0], e[1])]
    return addr[i] + 256 * e[2] + 4 * l


def gcost(g):
    tot = 0
    for row in R[g]:
        for h in (0, 32):
            banks, seen = {}, set()
            for e in row[h:h + 32]:
                s = -4 if e is None else slot(e)  # padding lanes: one shared trash slot
                if s not in seen:
                    seen.add(s)
                    banks[(s // 4) % 32] = banks.get((s // 4) % 32, 0) + 1
            tot += max(banks.values())
    return tot


cost = {g: gcost(g) for g in groups}
total = sum(cost.values())
print(f"{std} {rate} z={z}: {len(groups)} variable groups, {len(cgroups)} check groups; variable-pass LDS cycles "
      f"{total} (conflict-free {sum(2 * int(vd[g]) for g in groups)}); search '{mode}', {iters} swaps", flush=True)
rng = np.random.default_rng(2)
if mode == "chk":
    users, bydeg = {}, {}
    for g in groups:
        for row in R[g]:
            for e in row:
                if e is not None:
                    users.setdefault((e[0], e[1]), set()).add(g)
    for i, cg in enumerate(cgroups):
        for l in range(int(cv[cg])):
            bydeg.setdefault(deg[i], []).append((i, l))
else:
    bydeg = {}
    for g in groups:
        for l in np.nonzero(vmap[g] >= 0)[0]:
            bydeg.setdefault(int(vd[g]), []).append((g, int(l)))
keys = list(bydeg)
for it in range(1, iters + 1):
    lst = bydeg[keys[rng.integers(len(keys))]]
    a, b = lst[rng.integers(len(lst))], lst[rng.integers(len(lst))]
    if a == b:
        continue
    if mode == "chk":
        aff = users.get(a, set()) | users.get(b, set())
        place[a], place[b] = place[b], place[a]
    else:
        aff = {a[0], b[0]}
        for row_a, row_b in zip(R[a[0]], R[b[0]]):
            row_a[a[1]], row_b[b[1]] = row_b[b[1]], row_a[a[1]]
    new = {g: gcost(g) for g in aff}
    delta = sum(new.values()) - sum(cost[g] for g in aff)
    if delta <= 0:
        cost.update(new)
        total += delta
    elif mode == "chk":
        place[a], place[b] = place[b], place[a]
    else:
        for row_a, row_b in zip(R[a[0]], R[b[0]]):
            row_a[a[1]], row_b[b[1]] = row_b[b[1]], row_a[a[1]]
    if it % 50000 == 0:
        print(f"  {it} swaps: {total}", flush=True)
print(f"final {total}")
