"""Per-kernel totals from a rocprofv3 kernel trace (sqlite .db or *_kernel_trace.csv); --by-grid
splits a kernel's launches by grid size (e.g. the 1B-point encode vs the PCIe leg's 8M-point chunks)."""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def rows(path, by_grid=False):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e in c.execute("select name, start, end from kernels"):
            yield name, s, e
    else:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if by_grid:   # launches of one kernel at different sizes apart (grid = threads launched)
                name = "[grid %s] %s" % (r.get("Grid_Size_X", r.get("Grid_Size", "?")), name)
            yield name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])


def main(path, by_grid=False):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) + \
            glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = cands[0]
    agg = defaultdict(list)
    for n, s, e in rows(path, by_grid):
        agg[n].append(e - s)
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print("%8.3f ms total %5d calls %9.1f us avg  %s" % (sum(v) / 1e6, len(v), sum(v) / len(v) / 1e3, n[:90]))


if __name__ == "__main__":
    main(sys.argv[1], "--by-grid" in sys.argv[2:])
