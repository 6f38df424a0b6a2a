"""Summarises the alternating A/B runs of tools/gpu_lease.sh (ab step): one line per (library, round)
with the ms of every leg the detail records carry.  usage: python tools/show_ab.py gpurun_out/TAG_ab"""
import glob
import json
import re
import sys


def legs(d):
    out = {}
    if "ms_per_step" in d:
        out["z3"] = d["ms_per_step"]
    pj = d.get("pip_join") or {}
    if pj:
        out["join"] = pj["ms_per_step"]
        if "row_predicate" in pj:
            out["relate"] = pj["row_predicate"]["ms_per_step"]
    for k, v in (d.get("extra") or {}).items():
        if isinstance(v, dict) and "ms_per_step" in v:
            out[k] = v["ms_per_step"]
            if isinstance(v.get("device_output"), dict):
                out[k + "_dev"] = v["device_output"]["ms_per_step"]
    return out


def main(prefix):
    rows = []
    for f in sorted(glob.glob(prefix + "_*_*.detail.json")):
        m = re.match(re.escape(prefix) + r"_(.+)_(\d+)\.detail\.json$", f)
        if m:
            rows.append((m.group(1), int(m.group(2)), legs(json.load(open(f)))))
    keys = sorted({k for _, _, l in rows for k in l})
    print("lib round " + " ".join(keys))
    for lib, r, l in sorted(rows, key=lambda t: (t[1], t[0])):
        print(lib, r, " ".join("%.4f" % l[k] if k in l else "-" for k in keys))


if __name__ == "__main__":
    main(sys.argv[1])
