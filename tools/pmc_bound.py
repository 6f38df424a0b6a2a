"""Derived bound metrics of one kernel from rocprofv3 --pmc passes (gpu_lease.sh pmc:LEG):
  python tools/pmc_bound.py DIR PATTERN [FIRST COUNT]
DIR holds p0..pN (one counter group each); PATTERN selects the kernel by name; FIRST / COUNT pick that
kernel's dispatches (in order) when one run launches it for several cases.  Counters are summed over a
dispatch; GRBM_GUI_ACTIVE is summed over the 8 XCDs, the TA / TD / TCP *_sum counters over the 256 CUs,
SQ_* cycle counters over waves (quad-cycles, MI355X_MICROARCH.md)."""
import csv
import glob
import os
import sys
from collections import defaultdict

CUS, XCDS = 256, 8


def load(root, pattern, first=0, count=None):
    vals = defaultdict(list)   # counter -> per-dispatch values (in dispatch order)
    durs = []
    for d in sorted(glob.glob(os.path.join(root, "p*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        per = defaultdict(lambda: defaultdict(float))
        tim = {}
        for r in csv.DictReader(open(f)):
            if pattern not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            tim[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6   # ms
        ks = sorted(per)[first:first + count if count else None]
        for k in ks:
            for c, v in per[k].items():
                vals[c].append(v)
            durs.append(tim[k])
    return {c: sum(v) / len(v) for c, v in vals.items()}, (sum(durs) / len(durs) if durs else None)


def main():
    root, pat = sys.argv[1], sys.argv[2]
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    count = int(sys.argv[4]) if len(sys.argv) > 4 else None
    v, ms = load(root, pat, first, count)
    g = v.get("GRBM_GUI_ACTIVE")
    cyc = g / XCDS if g else None   # kernel cycles (per XCD)
    out = []
    if ms:
        out.append(("profiled dispatch time (ms, mean over passes)", "%.3f" % ms))
    if cyc and ms:
        out.append(("effective clock (GHz) = GRBM / 8 / time", "%.2f" % (cyc / (ms * 1e-3) / 1e9)))
    def frac(name, num, den):
        if num in v and den:
            out.append((name, "%.1f%%" % (100.0 * v[num] / den)))
    if "SQ_WAVE_CYCLES" in v:
        w = v["SQ_WAVE_CYCLES"]
        frac("waves waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES)", "SQ_WAIT_ANY", w)
        frac("issue-stalled (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)", "SQ_WAIT_INST_ANY", w)
        frac("issuing VALU (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES)", "SQ_ACTIVE_INST_VALU", w)
        frac("issuing VMEM (SQ_ACTIVE_INST_VMEM / SQ_WAVE_CYCLES)", "SQ_ACTIVE_INST_VMEM", w)
        frac("issuing LDS (SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES)", "SQ_ACTIVE_INST_LDS", w)
    if cyc:
        frac("TA busy (TA_TA_BUSY_sum / 256 CUs / cycles)", "TA_TA_BUSY_sum", CUS * cyc)
        frac("TD busy (TD_TD_BUSY_sum / 256 CUs / cycles)", "TD_TD_BUSY_sum", CUS * cyc)
        frac("TD stalled on the L1 (TD_TC_STALL_sum)", "TD_TC_STALL_sum", CUS * cyc)
        frac("L1 stalled on pending misses (TCP_PENDING_STALL_CYCLES_sum)", "TCP_PENDING_STALL_CYCLES_sum", CUS * cyc)
        if "SQ_BUSY_CYCLES" in v:
            out.append(("SQ busy cycles / kernel cycles (per XCD, 32 CUs)", "%.2f" % (v["SQ_BUSY_CYCLES"] / cyc / XCDS)))
    if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
        h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
        out.append(("L2 hits / misses", "%.3g / %.3g (hit rate %.1f%%)" % (h, m, 100 * h / max(1.0, h + m))))
    if "TCP_TCC_READ_REQ_sum" in v and "TCP_TCC_READ_REQ_LATENCY_sum" in v:
        out.append(("mean L1->L2 read latency (cycles)", "%.0f" % (v["TCP_TCC_READ_REQ_LATENCY_sum"] / max(1.0, v["TCP_TCC_READ_REQ_sum"]))))
    if "FETCH_SIZE" in v:
        out.append(("FETCH_SIZE (GB raw; x2 for 16-B streaming reads)", "%.3f" % (v["FETCH_SIZE"] * 1024 / 1e9)))
    if "WRITE_SIZE" in v:
        out.append(("WRITE_SIZE (GB)", "%.3f" % (v["WRITE_SIZE"] * 1024 / 1e9)))
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_WAVES"):
        if c in v:
            out.append((c, "%.4g" % v[c]))
    w = max(len(a) for a, _ in out) if out else 0
    print("kernel %s (dispatches %d..%s)" % (pat, first, "" if count is None else first + count - 1))
    for a, b in out:
        print("  %-*s  %s" % (w, a, b))


if __name__ == "__main__":
    main()
