"""Summarise rocprofv3 --pmc CSV passes: per kernel (name filter), mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def summarise(root, pattern):
    acc = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    dur = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if pattern not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            acc[r["Counter_Name"]][key] += float(r["Counter_Value"])
    out = {}
    for c, d in acc.items():
        out[c] = sum(d.values()) / len(d)
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1], sys.argv[2])
    for k in sorted(res):
        print("%-28s %.4g" % (k, res[k]))
