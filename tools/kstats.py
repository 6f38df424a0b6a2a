"""Per-kernel totals from a rocprofv3 kernel trace (sqlite .db or *_kernel_trace.csv)."""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e in c.execute("select name, start, end from kernels"):
            yield name, s, e
    else:
        for r in csv.DictReader(open(path)):
            yield r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])


def main(path):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) + \
            glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = cands[0]
    agg = defaultdict(list)
    for n, s, e in rows(path):
        agg[n].append(e - s)
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print("%8.3f ms total %5d calls %9.1f us avg  %s" % (sum(v) / 1e6, len(v), sum(v) / len(v) / 1e3, n[:90]))


if __name__ == "__main__":
    main(sys.argv[1])
