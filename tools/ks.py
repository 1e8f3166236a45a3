"""Per-kernel averages of rocprofv3 kernel_stats CSVs: python tools/ks.py a.csv [b.csv ...]"""
import csv
import sys
for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        nm = r["Name"].split("(")[0].split("::")[-1]
        print("  %-28s calls %5s avg %10.1f us  total %9.2f ms" % (nm[:28], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                                  float(r["TotalDurationNs"]) / 1e6))
