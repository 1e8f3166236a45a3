"""Launch gaps of a rocprofv3 --kernel-trace CSV: for the dispatches between
two kernel-name markers (default: every dispatch), the GPU-busy time (union of
kernel intervals), the idle time between consecutive kernels, and the largest
gaps with the kernels on either side.

usage: python tools/gap_report.py run_kernel_trace.csv [first-kernel-prefix]"""
import collections
import csv
import sys


def main(path, start_prefix=None):
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    if start_prefix:
        i0 = next((i for i, r in enumerate(rows) if r[2].startswith(start_prefix)), 0)
        rows = rows[i0:]
    busy, idle, gaps = 0, 0, []
    end = rows[0][0]
    for s, e, n in rows:
        if s > end:
            idle += s - end
            gaps.append((s - end, prev, n))
        busy += max(0, e - max(s, end))
        end = max(end, e)
        prev = n
    span = rows[-1][1] - rows[0][0]
    print(f"dispatches {len(rows)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {idle / 1e6:.3f} ms "
          f"({idle / span:.1%})")
    by = collections.defaultdict(lambda: [0, 0])
    for g, a, b in gaps:
        by[(a.split("<")[0], b.split("<")[0])][0] += g
        by[(a.split("<")[0], b.split("<")[0])][1] += 1
    print("idle by (previous kernel -> next kernel):")
    for k, (t, c) in sorted(by.items(), key=lambda x: -x[1][0])[:15]:
        print(f"  {t / 1e6:8.3f} ms  {c:6d} gaps  mean {t / c / 1e3:7.2f} us  {k[0]} -> {k[1]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
