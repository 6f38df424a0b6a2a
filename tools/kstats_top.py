"""Top kernels of a rocprofv3 --stats run: python tools/kstats_top.py DIR [N]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/*kernel_stats.csv")[0]
for r in list(csv.DictReader(open(f)))[:int(sys.argv[2]) if len(sys.argv) > 2 else 14]:
    print(r["Name"][:70].ljust(70), r["Calls"].rjust(5), "%9.3f" % (float(r["AverageNs"]) / 1e6),
          "%9.2f" % (float(r["TotalDurationNs"]) / 1e6))
