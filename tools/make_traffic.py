"""Per-launch HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes -> profiles/pmc_traffic.json.

usage: python tools/make_traffic.py PMC_DIR OUT_JSON [points] [join_points] [table_rows]

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  The read side is calibrated on known byte counts
(tools/traffic_probe.hip, profiles/r6/traffic_probe_pmc.txt): on gfx950 EVERY memory-side read request
is a 128-B line -- TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ for coalesced 16-B streams, whole-line gathers,
one 4-B word per line, and random 4-, 8- and 16-B gathers over a 4 GiB table alike -- while FETCH_SIZE
tallies 64 B per request, so it reports half the bytes for all of them (not only for wide streaming
reads).  The read bytes are therefore 32 n_32B + 64 n_64B + 128 n_128B from the TCC_EA0_RDREQ size
counters when that pass exists (`fetch_source` "rdreq_sizes"), else 2 x FETCH_SIZE, which the probe
shows to be the same for these access shapes.  WRITE_SIZE (64 B per 64-B write request) reads 16-B
streaming stores exactly (the probe's copy).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# bench name -> (kernel-name substring, unit count per launch key, algorithmic bytes per unit)
STREAMING = {
    "z3_index_key": ("k_z3_index_key<", "points", 34.0),
    "z3_invert": ("k_z3_invert<", "points", 32.0),
    "z2_index": ("k_z2_index<", "points", 24.0),
    "z2_invert": ("k_z2_invert<", "points", 24.0),
    "z3filter_scan": ("k_z3filter_mask_v", "points", 10.125),
    "xz2_index": ("k_xz2_index_v", "xz", 40.0),
    "xz3_index": ("k_xz3_index_v", "xz", 56.0),
    "query_scan_polygon": ("k_query_mask<true, false, 1>", "points", 16.125),
    "z3_histogram": ("k_z3_hist_lds<", "points", 24.0),
    "pip_relate": ("k_pip_relate", "points", 21.0),
    "sort_count": ("k_sort_count<", "rows", 10.0),
    "sort_pass_first": ("k_sort_pass<false, false", "rows", 26.0),
    "sort_pass": ("k_sort_pass<true, false", "rows", 32.0),
    "sort_local": ("k_sort_local<", "rows", 34.0),
}
# join step kernels and the points per dispatch: one direct pass per 2^31 points
JOIN_MODES = {"direct": (["k_pip_join_q<true", "k_pair_plan", "k_pair_move"], 1 << 31)}


def per_dispatch(root):
    """kernel name -> counter -> list of per-dispatch values (summed over the counter's instances)."""
    acc = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            key = (f, r["Dispatch_Id"])
            names[key] = r["Kernel_Name"]
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for key, cs in acc.items():
        for c, v in cs.items():
            out[names[key]][c].append(v)
    return out


def mean_for(d, sub, counter, largest=False):
    """Mean per dispatch of kernels whose name holds `sub`; largest=True keeps only the dispatches of
    the largest launches (e.g. the 1B-point encode, not the PCIe leg's 8M-point chunks of the same
    kernel): those within half of the largest value."""
    vals = [v for k, cs in d.items() if sub in k for v in cs.get(counter, [])]
    if largest and vals:
        top = max(vals)
        vals = [v for v in vals if v >= 0.5 * top]
    return sum(vals) / len(vals) if vals else None


def read_bytes(d, sub, largest=False):
    """(bytes read per dispatch, source): the TCC_EA0_RDREQ size counters when present, else 2 x FETCH_SIZE."""
    n128 = mean_for(d, sub, "TCC_EA0_RDREQ_128B_sum", largest)
    if n128 is not None:
        n64 = mean_for(d, sub, "TCC_EA0_RDREQ_64B_sum", largest) or 0.0
        n32 = mean_for(d, sub, "TCC_EA0_RDREQ_32B_sum", largest) or 0.0
        return 128.0 * n128 + 64.0 * n64 + 32.0 * n32, "rdreq_sizes"
    f = mean_for(d, sub, "FETCH_SIZE", largest)
    return (None, None) if f is None else (2.0 * f * 1024, "fetch_size_x2")


def main(root, out, points=1_000_000_000, join_points=1_000_000_000, table_rows=250_000_000):
    d = per_dispatch(root)
    res = {}
    for name, (sub, unit, alg) in STREAMING.items():
        f, w = mean_for(d, sub, "FETCH_SIZE", True), mean_for(d, sub, "WRITE_SIZE", True)
        fb, src = read_bytes(d, sub, True)
        if fb is None or w is None:
            continue
        n = points if unit == "points" else (table_rows if unit == "rows" else min(points, 100_000_000))
        wb = w * 1024
        res[name] = {"n": n, "kernel": sub, "bytes_per_launch": fb + wb, "fetch_bytes": fb, "write_bytes": wb,
                     "fetch_size_raw_kib": f, "write_size_kib": w, "algorithmic_bytes": alg * n,
                     "traffic_over_algorithmic": round((fb + wb) / (alg * n), 4), "fetch_source": src,
                     "correction": "read bytes = 128 B per TCC_EA0_RDREQ_128B request (= 2 x FETCH_SIZE on gfx950, "
                                   "calibrated by tools/traffic_probe.hip)"}
    for mode, (kernels, chunk) in JOIN_MODES.items():
        nchunks = -(-join_points // chunk)
        parts, total_raw, total = {}, 0.0, 0.0
        for k in kernels:
            f, w = mean_for(d, k, "FETCH_SIZE"), mean_for(d, k, "WRITE_SIZE")
            fb, src = read_bytes(d, k)
            if f is None or w is None or fb is None:
                continue
            parts[k] = {"fetch_size_raw_kib": f, "write_size_kib": w, "read_bytes": fb, "fetch_source": src}
            total_raw += (f + w) * 1024 * nchunks
            total += (fb + w * 1024) * nchunks
        if len(parts) == len(kernels):
            res["pip_join"] = {"n": join_points, "mode": mode, "kernels": parts, "dispatches": nchunks,
                               "bytes_per_launch": total, "bytes_raw": total_raw,
                               "note": "whole join step; reads = 128 B per memory-side read request, the index gathers "
                                       "included (every L2 miss fetches a whole 128-B line: tools/traffic_probe.hip); "
                                       "FETCH_SIZE + WRITE_SIZE uncorrected in bytes_raw"}
    # FP64 VALU work of the join (SQ_INSTS_VALU_FLOPS_FP64 pass), per launch
    fp = mean_for(d, "k_pip_join_q<true", "SQ_INSTS_VALU_FLOPS_FP64")
    if fp is not None:
        res["pip_join_fp64"] = {"n": join_points, "sq_insts_valu_flops_fp64": fp,
                                "note": "rocprofv3 SQ_INSTS_VALU_FLOPS_FP64 per dispatch of the direct join kernel"}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in res.items():
        if "bytes_per_launch" in v:
            print("%-14s %8.2f GB/launch" % (k, v["bytes_per_launch"] / 1e9))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], *(int(v) for v in a[2:]))
