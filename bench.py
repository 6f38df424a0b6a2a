"""Headline benchmark: Z3 encode points/s + st_contains join pairs/s on MI355X (BASELINE.json).

  python bench.py [--gpus N --steps K --warmup W]           (N > 1: launched by torch.distributed.run)

A step of the headline is one pass of Z3IndexKeySpace.toIndexKey's batch form (BinnedTime(week) +
Z3SFC.index) over the rank's resident 1B-point shard (BASELINE configs[1]); `value` = points of all
ranks / max-over-ranks time.  The st_contains join (configs[3]: 1B points x 3,200 county polygons,
polygon set broadcast over RCCL) is timed the same way and reported under "pip_join"; the remaining
hot-path kernels are reported under "extra".  Inputs are generated on the device (SplitMix64) before
the timed region; the CPU restatement (oracle/) is timed on a bounded sample as cpu_baseline.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from geomesa_amd.shard import all_reduce_scalar, gather_rows, shard_bounds  # noqa: E402

METRIC = "points/sec Z3 encode + point-in-polygon join pairs/sec at 1/2/4/8 MI355X"
SEED = 0x67656F6D65736121
T2020, T2021 = 1577836800000, 1609459200000
CONUS = (-125.0, 24.0, -66.0, 50.0)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6        # FP64 vector


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--points", type=int, default=1_000_000_000, help="points per GPU (Z3 encode)")
    p.add_argument("--join-points", type=int, default=1_000_000_000, help="points per GPU (join)")
    p.add_argument("--join-steps", type=int, default=5)
    p.add_argument("--no-extra", action="store_true")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=8.0)
    p.add_argument("--only", default="", help="comma list: z3,join,extra,table (profiling)")
    p.add_argument("--table-rows", type=int, default=250_000_000,
                   help="rows per GPU of the sorted-table leg (configs[2]: 2B rows over 8 GPUs)")
    p.add_argument("--join-mode", default="auto", choices=["auto", "direct"])
    p.add_argument("--cells-per-poly", type=int, default=0, help="join grid density (0 = library default)")
    p.add_argument("--join-grid", default="80x40", help="synthetic county grid (experiments)")
    p.add_argument("--no-gather", action="store_true", help="skip the join's result gather to rank 0")
    p.add_argument("--join-sorted", action="store_true", help="experiment: points pre-sorted by latitude")
    return p.parse_args()


class Dist:
    def __init__(self, ngpus):
        import torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # rehearsal knobs (never used by the driver's runs): GM_BENCH_DEVICE puts every rank on one GPU,
        # GM_BENCH_BACKEND=gloo runs the collectives through host memory, so the N > 1 paths can be
        # exercised on a one-GPU box
        if os.environ.get("GM_BENCH_DEVICE"):
            self.local = int(os.environ["GM_BENCH_DEVICE"])
        backend = os.environ.get("GM_BENCH_BACKEND", "nccl")
        torch.cuda.set_device(self.local)
        self.pg = None
        # a process group whenever torch.distributed.run launched us, even at world 1 (every RCCL branch
        # then runs with one rank: tests/test_gpu_rccl.py); a plain `python bench.py` has none
        if self.world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group(backend)
            self.pg = dist

    def barrier(self):
        import torch
        torch.cuda.synchronize()
        if self.pg:
            self.pg.barrier()
        torch.cuda.synchronize()

    def max(self, v):
        return all_reduce_scalar(self.pg, v, "max")

    def sum(self, v):
        return all_reduce_scalar(self.pg, v, "sum")


def box_copy_gbs(dist, src, ctx):
    """HBM rate (read + write bytes / time) of a 4 GB device-to-device copy on this rank's GPU, the
    slowest rank's, best of 5: the box's own streaming ceiling.  The copy is gm_device_copy (16 B per
    lane, four vectors in flight per lane, non-temporal loads and stores -- the encode kernels' access
    shape), timed with HIP events on the context stream; torch's byte copy_ had run slower than the
    encode kernel itself, so a frac_of_box_copy above 1 meant nothing."""
    import torch
    from geomesa_amd import _lib
    n = min(src.numel() * src.element_size(), 4 << 30) // 16 * 16
    a = src.view(torch.uint8)[:n]
    b = torch.empty(n, dtype=torch.uint8, device=src.device)
    best = None
    for _ in range(6):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        _lib.check(ctx.lib.gm_device_copy(ctx.handle, _lib.ptr(b), _lib.ptr(a), n), "gm_device_copy")
        e.record()
        torch.cuda.synchronize()
        best = s.elapsed_time(e) if best is None else min(best, s.elapsed_time(e))
    del b
    return all_reduce_scalar(dist.pg, 2.0 * n / (best * 1e-3) / 1e9, "min")


def timed(dist, fn, steps, warmup):
    """Barrier + sync on both sides; HIP events on the stream the kernels run on; max over ranks."""
    import torch
    for _ in range(warmup):
        fn()
    dist.barrier()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / steps
    dist.barrier()
    return dist.max(ms)


def gen_points(ctx, n, base, box, x, y, t):
    from geomesa_amd import _lib
    _lib.check(ctx.lib.gm_gen_points(ctx.handle, SEED, n, base, box[0], box[2], box[1], box[3], T2020, T2021,
                                     _lib.ptr(x), _lib.ptr(y), _lib.ptr(t)), "gm_gen_points")


def load_pmc(name, n):
    """Per-launch HBM traffic from a committed rocprofv3 PMC summary (profiles/), if it matches n."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))[name]
        if int(d["n"]) == int(n):
            return float(d["bytes_per_launch"])
    except Exception:
        pass
    return None


def load_profile(name, n):
    """A committed per-launch PMC record (profiles/pmc_traffic.json) when it was taken at this size."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))[name]
        return d if int(d["n"]) == int(n) else None
    except Exception:
        return None


def roofline(bytes_per_launch, ms, traffic=None):
    gbs = bytes_per_launch / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic}


# ------------------------------------------------------------------------------ CPU baselines

def cpu_threads():
    """The CPUs this process can actually use: min(affinity set, cgroup CPU quota) -- on the GPU boxes
    a 16-CPU quota over a 256-CPU machine (BASELINE.md:38-43: the CPU baseline runs at 1 thread and
    at the usable core count).  The machine's logical count is reported beside it (cpu_info)."""
    info = cpu_info()
    n = info["affinity_cpus"] or os.cpu_count() or 1
    if info["cgroup_cpu_quota"]:
        n = min(n, max(1, int(info["cgroup_cpu_quota"])))
    return max(1, n)


def cpu_info():
    """The CPU the baselines ran on: model, logical CPUs, this process's affinity and cgroup quota."""
    info = {"cpu_model": None, "logical_cpus": os.cpu_count(), "affinity_cpus": None, "cgroup_cpu_quota": None}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["cpu_model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q and q[0] != "max":
            info["cgroup_cpu_quota"] = round(int(q[0]) / int(q[1]), 2)
    except (OSError, ValueError, IndexError):
        pass
    return info


def timed_threads(nt, seconds, call):
    """Runs call(k, nt) (one unit of thread k's work; returns units done) on nt threads for about
    `seconds`; returns (units per second, seconds, units)."""
    done = [0] * nt
    stop = time.time() + seconds

    def work(k):
        while time.time() < stop:
            done[k] += call(k, nt)
    th = [threading.Thread(target=work, args=(k,)) for k in range(nt)]
    t0 = time.time()
    for h in th:
        h.start()
    for h in th:
        h.join()
    dt = time.time() - t0
    return sum(done) / dt, dt, sum(done)


def cpu_z3_baseline(seconds, sample):
    """The oracle on the host cores at 1 thread and at nproc threads, over a strided sample of the GPU
    run's own points (each thread keys its slice of the sample, repeatedly); the sample's keys are
    also compared with what the GPU wrote for them (full-size parity, strided)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    x, y, t, gb, gz, stride = sample
    per = len(x)
    ob, oz, ost = O.z3_index_key_batch(x, y, t)
    bad = int(((ob != gb) | (oz != gz) | (ost != 0)).sum())
    L = O.lib()
    b = np.empty(per, np.int16); z = np.empty(per, np.int64); st = np.empty(per, np.uint8)

    def call(k, nt):
        lo, hi = per * k // nt, per * (k + 1) // nt
        L.gmo_z3_index_key_batch(1, O._p(x[lo:hi]), O._p(y[lo:hi]), O._p(t[lo:hi]), hi - lo, 0, O._p(b[lo:hi]),
                                 O._p(z[lo:hi]), O._p(st[lo:hi]))
        return hi - lo
    v1, dt1, n1 = timed_threads(1, seconds / 2, call)
    nt = cpu_threads()
    vn, dtn, nn = timed_threads(nt, seconds / 2, call)
    return {"value": vn, "unit": "points/s", "cores": nt, "kind": "port",
            "threads_1": {"value": v1, "seconds": round(dt1, 2), "points": n1},
            "host": cpu_info(),
            "sample": "C restatement (oracle gmo_z3_index_key_batch, week) over every %d-th point of the GPU "
                      "run (%d points), each of %d threads keying its slice repeatedly for %.1f s (%d points); "
                      "1 thread: %.1f s" % (stride, per, nt, dtn, nn, dt1),
            "parity_sample": {"points": per, "stride": stride, "mismatches": bad,
                              "note": "bin / z of the strided sample of the 1B-point GPU run against the oracle"}}


def cpu_join_baseline(seconds, ps, sample=None):
    """The oracle's join on the host cores at 1 thread and at nproc threads; with `sample` (every
    stride-th point of the GPU run and the GPU's pairs for those points) it also reports full-size
    parity of the strided sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from geomesa_amd.join import synthetic_points
    nt = cpu_threads()
    op = O.OraclePolySet(*ps.to_arrays())
    parity = None
    if sample is not None:
        sx, sy, stride, gpu_pairs = sample
        opt, opl = op.join(sx, sy, nthreads=nt)
        exp = np.stack([opt.astype(np.int64), opl.astype(np.int64)], 1)
        exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
        got = gpu_pairs[np.lexsort((gpu_pairs[:, 1], gpu_pairs[:, 0]))]
        parity = {"points": len(sx), "stride": stride, "pairs": len(exp), "gpu_pairs": len(got),
                  "equal": bool(len(exp) == len(got) and np.array_equal(exp, got)),
                  "note": "(point, polygon) pairs of every stride-th point of the 1B-point GPU join against the oracle"}
    px, py = synthetic_points(20_000, seed=SEED + 5)
    t0 = time.time()
    op.join(px[:2000], py[:2000], nthreads=1)
    est = max(time.time() - t0, 1e-4) / 2000   # seconds per point on one thread

    def run(threads, secs):
        n = int(min(50_000_000, max(20_000, secs * threads / est)))
        qx, qy = synthetic_points(n, seed=SEED + 5)
        t1 = time.time()
        pt, _ = op.join(qx, qy, nthreads=threads)
        dt = time.time() - t1
        return n * ps.n_polys / dt, n, dt, len(pt)
    v1, n1, dt1, m1 = run(1, seconds / 2)
    vn, nn, dtn, mn = run(nt, seconds / 2)
    out = {"value": vn, "unit": "pairs/s", "cores": nt, "kind": "port",
           "threads_1": {"value": v1, "points": n1, "seconds": round(dt1, 2)},
           "host": cpu_info(),
           "sample": "%d CONUS points x %d polygons, C restatement (grid candidates + JTS contains per "
                     "pair, %d pthreads): %.2f s, %d matches; 1 thread: %d points in %.2f s"
                     % (nn, ps.n_polys, nt, dtn, mn, n1, dt1)}
    if parity is not None:
        out["parity_sample"] = parity
    return out


def range_digest(offs, rr):
    """sha256 over the per-query offsets and every range's (lower, upper, contained)."""
    import hashlib
    h = hashlib.sha256(np.ascontiguousarray(offs, np.int64).tobytes())
    for f in ("lower", "upper", "contained"):
        h.update(np.ascontiguousarray(rr[f]).tobytes())
    return h.hexdigest()[:16]


def cpu_ranges_baseline(kind, q, t, max_ranges, gpu_ms, nq, gpu_lists=None, dev_ms=None):
    """The oracle's range decomposition of the same queries on the host's cores (all of them: the
    nodes-checked total is the work measure of the GPU batch too, SURVEY 8(d) ranges() row).  With the
    GPU's gathered (offsets, ranges), every query's merged list is compared with the oracle's
    (lower, upper, contained; XZ2SFC.scala:146-252, XZ3SFC.scala:156-262, ZN.scala:110-242)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    nt = cpu_threads()
    t0 = time.time()
    r, nodes = O.ranges_batch(kind, q, t, max_ranges=max_ranges, nthreads=nt)
    dt = time.time() - t0
    out = {"cpu_baseline": {"value": nq / dt, "unit": "queries/s", "cores": nt, "kind": "port",
                            "sample": "all %d queries through the C restatement (%d pthreads): %.2f s, %d ranges"
                                      % (nq, nt, dt, r)},
           "nodes_checked": nodes, "nodes_checked_per_s": nodes / (gpu_ms * 1e-3),
           "cpu_ranges": r}
    if dev_ms:   # the same work measure over the device-output time (ranges left in HBM)
        out["nodes_checked_per_s_device_output"] = nodes / (dev_ms * 1e-3)
    if gpu_lists is not None:
        _, _, coffs, crr = O.ranges_batch(kind, q, t, max_ranges=max_ranges, nthreads=nt, lists=True)
        goffs, grr = gpu_lists
        grr = grr[:int(goffs[-1])]
        eq = bool(np.array_equal(coffs, goffs) and
                  all(np.array_equal(crr[f], grr[f]) for f in ("lower", "upper", "contained")))
        out["parity"] = {"queries": nq, "ranges": int(coffs[-1]), "ranges_equal": eq,
                         "oracle_digest": range_digest(coffs, crr), "gpu_digest": range_digest(goffs, grr),
                         "note": "every query's merged range list (lower, upper, contained) from the GPU batch "
                                 "against the oracle's, all queries"}
    return out


def pcie_encode(dist, ctx, x, y, t, z_ref, n=64 << 20, chunk=8 << 20, reps=3):
    """Z3 key encode of host-resident columns: per chunk an H2D copy of x, y, t on one copy stream,
    the kernel on the compute stream, the bin / z D2H on a second copy stream, three device buffers
    in a ring -- so chunk k+1's H2D, chunk k's kernel and chunk k-1's D2H run at once (PCIe is
    full duplex: the bound is the 24 B/point H2D, not the 34 B/point sum)."""
    import torch
    from geomesa_amd import _lib
    n = min(n, x.numel())
    hx, hy, ht = (v[:n].cpu().pin_memory() for v in (x, y, t))
    hb = torch.empty(n, dtype=torch.int16).pin_memory()
    hz = torch.empty(n, dtype=torch.int64).pin_memory()
    dev = x.device
    NB = 3
    bufs = [dict(x=torch.empty(chunk, dtype=torch.float64, device=dev), y=torch.empty(chunk, dtype=torch.float64, device=dev),
                 t=torch.empty(chunk, dtype=torch.int64, device=dev), b=torch.empty(chunk, dtype=torch.int16, device=dev),
                 z=torch.empty(chunk, dtype=torch.int64, device=dev)) for _ in range(NB)]
    comp = torch.cuda.current_stream(dev)
    h2d, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    P = _lib.ptr

    def run():
        outs = []
        for k, c0 in enumerate(range(0, n, chunk)):
            m = min(chunk, n - c0)
            bf = bufs[k % NB]
            with torch.cuda.stream(h2d):
                if k >= NB:
                    h2d.wait_event(outs[k - NB])    # the buffer's last D2H (after its kernel) is done
                bf["x"][:m].copy_(hx[c0:c0 + m], non_blocking=True)
                bf["y"][:m].copy_(hy[c0:c0 + m], non_blocking=True)
                bf["t"][:m].copy_(ht[c0:c0 + m], non_blocking=True)
                e_in = torch.cuda.Event()
                e_in.record(h2d)
            comp.wait_event(e_in)
            _lib.check(ctx.lib.gm_z3_index_key(ctx.handle, P(bf["x"]), P(bf["y"]), P(bf["t"]), m, 1, 0, P(bf["b"]),
                                               P(bf["z"]), None, None), "gm_z3_index_key")
            e_k = torch.cuda.Event()
            e_k.record(comp)
            with torch.cuda.stream(d2h):
                d2h.wait_event(e_k)
                hb[c0:c0 + m].copy_(bf["b"][:m], non_blocking=True)
                hz[c0:c0 + m].copy_(bf["z"][:m], non_blocking=True)
                e_out = torch.cuda.Event()
                e_out.record(d2h)
            outs.append(e_out)
        torch.cuda.synchronize(dev)
    run()
    dist.barrier()
    t0 = time.time()
    for _ in range(reps):
        run()
    dist.barrier()
    dt = dist.max((time.time() - t0) / reps)
    ok = bool(torch.equal(hz, z_ref[:n].cpu()))   # same keys as the resident-column run
    return {"value": n * dist.world / dt, "unit": "points/s", "ms_per_step": dt * 1e3, "points_per_gpu": n,
            "pcie_gbps": 34.0 * n / dt / 1e9, "h2d_gbps": 24.0 * n / dt / 1e9, "checked": ok,
            "note": "PCIe-inclusive rate (host columns in pinned memory, 24 B/point in + 10 B/point out, "
                    "8M-point chunks in a ring of three device buffers: H2D on one copy stream, D2H on "
                    "another, so both directions and the kernel overlap); never `value`"}


def _lib_check(rc):
    from geomesa_amd import _lib
    _lib.check(rc, "batched ranges (device output)")


def ranges_batch(dist, fn, args, n_local, nq, reps=3):
    """One batched-ranges entry point over this rank's block of queries, then the gather of every
    rank's offsets + ranges to rank 0; wall time per batch (barrier on both sides, max over ranks)."""
    from geomesa_amd import ranges as R
    from geomesa_amd.shard import gather_ranges
    offs, rr, _ = R.call_raw(fn, args, n_local, max(n_local, 1) * 256, pinned=True)
    cap = int(offs[-1]) + 1024
    res = {}

    def step():
        o, r, _ = R.call_raw(fn, args, n_local, cap, pinned=True)
        g = gather_ranges(dist.pg, o, r[:int(o[-1])])
        res["n"] = int(g[0][-1]) if g is not None else -1
        res["g"] = g
    step()
    dist.barrier()
    t0 = time.time()
    for _ in range(reps):
        step()
    dist.barrier()
    dt = dist.max((time.time() - t0) / reps)
    # the last batch's gathered lists (views of the reused pinned output: copied out, untimed)
    g = res.pop("g")
    res["lists"] = (np.array(g[0]), np.array(g[1])) if g is not None else None
    # the same call writing into HBM (the ranges feed a device-side seek such as gm_key_range_scan):
    # no D2H copy of the ranges, no gather; per rank, max over ranks
    import torch
    dout = torch.empty(max(cap, 1) * R.RANGE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    offd = np.zeros(n_local + 1, np.int64)
    qst = np.zeros(max(n_local, 1), np.int32)
    needed = ctypes.c_int64()

    def dev_step():
        _lib_check(fn(*args, offd.ctypes.data, dout.data_ptr(), cap, ctypes.byref(needed), qst.ctypes.data))
    dev_step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.time()
    for _ in range(reps):
        dev_step()
    torch.cuda.synchronize()
    dist.barrier()
    ddt = dist.max((time.time() - t0) / reps)
    same = bool(np.array_equal(offd, offs)) if dist.world == 1 else None
    del dout
    return {"value": nq / dt, "unit": "queries/s", "ms_per_step": dt * 1e3, "ranges": res["n"],
            "device_output": {"ms_per_step": ddt * 1e3, "queries_per_s": nq / ddt, "offsets_equal": same,
                              "note": "ranges written into HBM (device-side consumer), windows H2D included"}}, res["lists"]


def sort_bytes(b, z, n, last):
    """Algorithmic bytes of gm_sort_keys over n unsharded rows, for the path the library reports
    (GM_PARAM_SORT_LAST: digit passes, + 256 when the runs of equal prefixes were ranked locally):
    the read that counts every pass's digits and takes the exact varying bits (10 B/row; the digits are
    planned from a 65,536-row sample, and a plan the exact bits change costs a second count read, which
    the bench's keys never need); the first pass reads the columns (10 B) and writes 16-B records
    {z, row, bin}, every later pass reads and writes records (32 B); then the local ranking reads the
    records and writes z, bin and the 8-B permutation (16 + 18 B), or the last digit pass writes those
    itself (18 B instead of 16).  Returns (bytes, passes, path)."""
    local = last >= 256
    npass = last - 256 if local else last
    total = 10.0 * n
    if npass:
        total += (10.0 + 16.0 + 32.0 * (npass - 1)) * n
    if local:
        total += 34.0 * n
        return total, npass, "one-sweep prefix passes + local ranks"
    total += 2.0 * n if npass else 0.0
    return total, npass, "one-sweep digit passes"


# Chip-wide access rates measured by tools/gather_probe.hip on MI355X (profiles/r2_gather_probe*.log:
# 2^30 accesses per launch, every CU busy): coalesced 16-B stream, a divergent 4/16-B gather from a
# table resident in L2 (1-4 MB), one that misses L2 (64 MB Infinity-Cache-resident to 1 GB tables:
# 56-59 G/s either way), and 8 lanes reading one random 128-B line together.
PROBE_STREAM_GBS, PROBE_L2_GPS, PROBE_FAR_GPS, PROBE_LINE_GPS = 6313.0, 270.0, 57.0, 14.3


def gather_model(census, points, pairs, ms):
    """The join's gather roofline: its lookups priced at the probe rates, per
    launch, from the lookup census of the same points.  Terms: the point stream and the pair writes
    (HBM), the coarse-table gathers (L2-resident table; points in EMPTY coarse blocks are answered by
    the LDS bitmap), the fine-word, line-entry and inline-fallback gathers (beyond L2: the fine table
    is ~210 MB), and the blob walks (~1.5 lines each at the shared-line rate).  frac = model / measured:
    how close the kernel is to what its gathers allow when every term runs back to back on the
    vector-memory path (the bound the r3 PMC named: TD busy > 90%)."""
    c = census
    far = c["fine"] + c["fine_line"] + c["inline_fallback"]
    blobs = c["fine_compact"] + c["fine_generic"] + c["line_fallback"] + c["inline_fallback"]
    terms = {"stream_ms": 16.0 * points / (PROBE_STREAM_GBS * 1e9) * 1e3,
             "pair_writes_ms": 12.0 * pairs / (PROBE_STREAM_GBS * 1e9) * 1e3,
             "coarse_l2_gathers_ms": c["coarse_gather"] / (PROBE_L2_GPS * 1e9) * 1e3,
             "beyond_l2_gathers_ms": far / (PROBE_FAR_GPS * 1e9) * 1e3,
             "blob_lines_ms": 1.5 * blobs / (PROBE_LINE_GPS * 1e9) * 1e3}
    model = sum(terms.values())
    return dict({k: round(v, 3) for k, v in terms.items()}, model_ms=round(model, 3), measured_ms=round(ms, 3),
                frac=round(model / ms, 4), counts={"coarse_gathers": c["coarse_gather"], "beyond_l2_gathers": far,
                                                   "blob_walks": blobs},
                rates="probe: stream %.0f GB/s, L2 gather %.0f G/s, beyond-L2 gather %.0f G/s, 128-B lines %.1f G/s"
                      % (PROBE_STREAM_GBS, PROBE_L2_GPS, PROBE_FAR_GPS, PROBE_LINE_GPS))


def scan_parity(dist, a, mask, n, check, stride_rows=2_000_000, max_matches=200_000):
    """Oracle sample of a full-size filter scan (rank 0, untimed): the mask bit (bit r & 63 of word
    r >> 6) of every stride-th row against the oracle's answer for those rows, plus the first
    `max_matches` rows the GPU marked as matches (a strided sample sees few of the rare matches).
    `check(rows)` maps a device int64 row tensor to the oracle's numpy bool answer."""
    if dist.rank != 0 or a.no_cpu:
        return None
    import torch
    stride = max(1, n // stride_rows)
    rows = torch.arange(0, n, stride, device=mask.device, dtype=torch.int64)
    got = (((mask[rows >> 6] >> (rows & 63)) & 1) != 0).cpu().numpy()
    exp = np.asarray(check(rows), bool)
    bit = torch.arange(64, device=mask.device, dtype=torch.int64)
    nzw = torch.nonzero(mask[:(n + 63) // 64]).flatten()[:max_matches]
    mb = ((mask[nzw].view(-1, 1) >> bit) & 1) != 0
    mrows = (nzw.view(-1, 1) * 64 + bit)[mb]
    mrows = mrows[mrows < n][:max_matches]
    mexp = np.asarray(check(mrows), bool) if mrows.numel() else np.zeros(0, bool)
    return {"rows": int(len(got)), "stride": stride, "sample_matches": int(exp.sum()),
            "gpu_matches_checked": int(len(mexp)), "false_positives": int((~mexp).sum()),
            "mismatches": int((got != exp).sum()) + int((~mexp).sum()),
            "note": "oracle (C restatement) on every stride-th row and on the first GPU matches of the full-size run"}


def gather_pairs(dist, ptids, plids, k, id_base, n_polys):
    """Result gather of the join, reported beside the sharded result the step leaves
    (the reference's join leaves its pairs in the RDD's partitions, GeoMesaJoinRelation.scala:41-91;
    ms_per_step is that placement).  Two wire formats to rank 0 over RCCL point-to-point: the full
    12-B pairs (shard.gather_rows) and the compact 6-B form (4-B shard-local row + 2-B polygon,
    shard.gather_pairs_compact, expanded on rank 0).  Each: measured ms (max over ranks), bytes on the
    wire, and the model estimate (largest peer's bytes over one ~153 GB/s xGMI link, or rank 0's HBM
    writes).  Never part of ms_per_step.  A failure is reported, not raised, so the scaling line
    survives it."""
    import torch
    from geomesa_amd.shard import gather_estimate_ms, gather_pairs_compact, gather_rows
    full_b = [12 * int(v) for v in all_gather_ints(dist, k)]
    # the compact format's bytes as gather_pairs_compact decides them: 6 B per pair only while every rank's
    # rows span < 2^32 and there are at most 65,536 polygons (else it sends the full 12-B pairs)
    span = int((ptids[:k].max() - id_base).item()) + 1 if k else 0
    fits = all(v == 1 for v in all_gather_ints(dist, int(span <= (1 << 32))))
    comp_b = [(6 if (n_polys <= 65536 and fits) else 12) * v // 12 for v in full_b]
    out = {"placement": "ms_per_step leaves the pairs sharded on their ranks (the reference's RDD partitions)",
           "est_ms_full": round(gather_estimate_ms(full_b), 3), "est_ms_compact": round(gather_estimate_ms(comp_b), 3),
           "bytes_full": sum(full_b[1:]), "bytes_compact": sum(comp_b[1:])}
    if dist.pg is None:   # one rank: the pairs already sit on rank 0, nothing moves
        out.update(noop=True, ms=0.0, bytes=0, pairs_on_rank0=int(k))
        return out
    try:
        dist.barrier()
        t0 = time.time()
        g = gather_rows(dist.pg, [ptids[:k], plids[:k]])
        torch.cuda.synchronize()
        ms = dist.max((time.time() - t0) * 1e3)
        n = int(g[0].numel()) if g is not None else 0
        del g
        torch.cuda.empty_cache()
        dist.barrier()
        t0 = time.time()
        gc, wire = gather_pairs_compact(dist.pg, ptids[:k], plids[:k], id_base, n_polys)
        out.update(bytes_compact=sum(wire[1:]), est_ms_compact=round(gather_estimate_ms(wire), 3))   # as sent
        torch.cuda.synchronize()
        msc = dist.max((time.time() - t0) * 1e3)
        nc = int(gc[0].numel()) if gc is not None else 0
        del gc
        torch.cuda.empty_cache()
        out.update(ms=ms, pairs_on_rank0=n if dist.rank == 0 else None, bytes=sum(full_b[1:]),
                   ms_compact=msc, pairs_on_rank0_compact=nc if dist.rank == 0 else None,
                   how="all_gather of counts, then batched point-to-point receives of exact sizes into rank 0's "
                       "output slices (RCCL send/recv over xGMI); compact: 6 B per pair on the wire, expanded on rank 0")
        return out
    except Exception as e:  # noqa: BLE001 -- reported in the JSON line
        out["error"] = repr(e)[:200]
        return out


def bench_table(a, dist, ctx, b, z):
    """configs[2]: a Z3 table range-sharded over the GPUs (2B rows over 8 GPUs = 250M per GPU).
    sort_keys: one gm_sort_keys of the rank's rows into table order.  table_ingest: the partitioned
    table built from the rank's rows (local sort, splitters, all-to-all by key range, slice sort).
    table_query: the configs[2] bbox + during query over the whole table -- ranges clipped to each
    slice, gm_key_range_scan (seek + Z3Filter), global ids gathered to rank 0."""
    import ctypes
    import torch
    from geomesa_amd import _lib
    from geomesa_amd import filters as F
    from geomesa_amd.keyspace import Z3IndexKeySpace, during
    from geomesa_amd.table import key_ranges
    NT = min(a.table_rows, b.numel())
    lib, h, P = ctx.lib, ctx.handle, _lib.ptr
    bs, zs = b[:NT], z[:NT]
    ob, oz = torch.empty_like(bs), torch.empty_like(zs)
    perm = torch.empty(NT, dtype=torch.int64, device=zs.device)

    def sort_step():
        _lib.check(lib.gm_sort_keys(h, None, P(bs), P(zs), NT, None, P(ob), P(oz), P(perm)), "gm_sort_keys")
    ms_sort = timed(dist, sort_step, 3, 1)
    sbytes, npass, spath = sort_bytes(bs, zs, NT, ctx.get_param(_lib.GM_PARAM_SORT_LAST))
    del ob, oz, perm
    # the key-range partitioned table (configs[2]): every rank keys its own rows, the ranks sample
    # splitters and exchange rows by key range (one all-to-all over RCCL), each sorts its slice
    from geomesa_amd.table import PartitionedZ3Table
    ks = Z3IndexKeySpace()
    holder = {}

    def ingest_step():
        holder.pop("t", None)
        # ids = the rank's first global row: rows travel as 4-B rows and map back through the senders' bases
        holder["t"] = PartitionedZ3Table(dist.pg, bs, zs, dist.rank * NT)
    ms_ingest = timed(dist, ingest_step, 1, 1)
    pt = holder["t"]
    # the partition pass of an N = 8 ingest on this rank's rows (7 splitters from its own key sample), timed
    # at every world size: at N > 1 it is one of the ingest's phases, at N = 1 the ingest has none
    from geomesa_amd import shard as S
    s_hi, s_lo = S.sample_keys(ctx, None, bs, zs, 1024)
    o = np.lexsort((s_lo, s_hi))
    pick = o[(np.arange(1, 8) * len(o)) // 8]
    sp8 = (s_hi[pick].copy(), s_lo[pick].copy())
    prt = {}

    def part_step():
        prt["cols"], prt["counts"] = S.partition_rows(ctx, None, bs, zs, *sp8, id_base=0, rows=True)
    ms_part = timed(dist, part_step, 3, 1)
    part_counts = prt["counts"]
    del prt
    phases = {k: (round(dist.max(v), 3) if isinstance(v, float) else v) for k, v in pt.timing.items()}
    slice_rows = [int(v) for v in (all_gather_ints(dist, pt.n))]
    v = ks.get_index_values([(-10, 35, 30, 60)], [during(1590969600000, 1591617600000)])
    t0 = time.time()
    sr = ks.get_ranges(v)
    plan_ms = (time.time() - t0) * 1e3
    arr, nr = key_ranges(sr)
    fb = F.serialize_to_bytes(F.Z3Filter.from_values(v))
    res = {}

    def query_step():
        ids, nm, ns, ncl = pt.scan(sr, fb)       # clip to the slice, seek + Z3Filter, global ids
        g = gather_rows(dist.pg, [ids])           # results to rank 0
        res.update(nm=nm, ns=ns, ncl=ncl, n0=int(g[0].numel()) if g is not None else -1)
    ms_scan = timed(dist, query_step, 10, 2)
    matches, scanned = dist.sum(res["nm"]), dist.sum(res["ns"])
    # the same query as a full scan of every rank's own unsorted rows: bin in the query's bins AND
    # Z3Filter.inBounds (ranges() covers the query box and the filter passes epochs outside
    # [minEpoch, maxEpoch], Z3Filter.scala:45-62, Z3IndexKeySpace.scala:196-238), global ids gathered
    # to rank 0 and compared as sets with the seek-and-filter result (untimed).  The full scan is the
    # oracle's (the C restatement, every row of the rank, chunked over the host threads); with --no-cpu
    # it is the library's own gm_z3filter_scan instead
    ids, nm, _, _ = pt.scan(sr, fb)
    got = gather_rows(dist.pg, [ids])
    br = np.asarray(ks.bin_ranges(v), np.int16).reshape(-1)
    if not a.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        from concurrent.futures import ThreadPoolExecutor
        hb, hz = bs.cpu().numpy(), zs.cpu().numpy()
        nt = cpu_threads()
        step = (NT + nt - 1) // nt
        with ThreadPoolExecutor(nt) as ex:   # ctypes drops the GIL inside the C call
            parts = list(ex.map(lambda k: np.nonzero(O.z3filter_scan(fb, br, hb[k:k + step], hz[k:k + step]))[0] + k,
                                range(0, NT, step)))
        fids = torch.as_tensor(np.concatenate(parts).astype(np.int64), device=zs.device)
        del hb, hz, parts
        how = "the oracle's z3filter_scan (C restatement) over every rank's unsorted rows"
    else:
        fbuf = (ctypes.c_uint8 * len(fb)).from_buffer_copy(fb)
        fmask = torch.empty((NT + 63) // 64, dtype=torch.int64, device=zs.device)
        fn = ctypes.c_int64()
        _lib.check(lib.gm_z3filter_scan(h, fbuf, len(fb), br.ctypes.data, len(br) // 2, P(bs), P(zs), NT, P(fmask),
                                        None, 0, ctypes.byref(fn)), "gm_z3filter_scan")
        fids = torch.empty(max(1, fn.value), dtype=torch.int64, device=zs.device)
        _lib.check(lib.gm_z3filter_scan(h, fbuf, len(fb), br.ctypes.data, len(br) // 2, P(bs), P(zs), NT, P(fmask),
                                        P(fids), fids.numel(), ctypes.byref(fn)), "gm_z3filter_scan")
        fids = fids[:fn.value]
        del fmask
        how = "gm_z3filter_scan (bin ranges + Z3Filter.inBounds) over every rank's unsorted rows"
    full = gather_rows(dist.pg, [fids + dist.rank * NT])
    qparity = None
    if dist.rank == 0:
        a_ids = np.sort(got[0].cpu().numpy()) if got is not None else np.zeros(0, np.int64)
        b_ids = np.sort(full[0].cpu().numpy()) if full is not None else np.zeros(0, np.int64)
        qparity = {"seek_ids": int(len(a_ids)), "full_scan_ids": int(len(b_ids)),
                   "ids_equal": bool(np.array_equal(a_ids, b_ids)),
                   "mismatches": int(len(np.setxor1d(a_ids, b_ids))),
                   "note": "ids of the range seek + Z3Filter over the partitioned table against " + how}
    del fids, got, full
    del holder, pt
    return {
        "sort_keys": {"value": NT * dist.world / (ms_sort * 1e-3), "unit": "rows/s", "ms_per_step": ms_sort,
                      "rows_per_gpu": NT, "digit_passes": npass, "path": spath,
                      "roofline": dict(roofline(sbytes, ms_sort), bytes_per_unit=round(sbytes / NT, 2),
                                       kernel="gm_sort_keys (all launches of one sort)",
                                       # against the compulsory bytes alone: the key columns read once
                                       # (bin 2 + z 8) and the sorted columns + 8-B permutation written once
                                       frac_compulsory=round(28.0 * NT / (ms_sort * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                       compulsory_bytes_per_unit=28),
                      "note": "stable sort of (bin, z) into table byte order (ingest side): one-sweep digit passes "
                              "(look-back, 16-B records) over the top ~log2(n) - 1 varying key bits, then every run of "
                              "equal prefixes ranked by full key in LDS (8-bit digit passes over every varying byte when "
                              "a run exceeds 256 rows); bytes: see sort_bytes"},
        "table_partition": {"value": NT * dist.world / (ms_part * 1e-3), "unit": "rows/s", "ms_per_step": ms_part,
                            "rows_per_gpu": NT, "destinations": 8, "rows_per_destination": part_counts,
                            # count read (bin 2 + z 8) + scatter read (10) + writes (bin 2 + z 8 + 4-B row)
                            "roofline": dict(roofline(34.0 * NT, ms_part), bytes_per_unit=34,
                                             kernel="gm_key_partition (count + scan + scatter)"),
                            "note": "gm_key_partition of the rank's unsorted rows into 8 key ranges (7 splitters from "
                                    "its own key sample): the per-rank partition pass of an N = 8 ingest"},
        "table_ingest": {"value": NT * dist.world / (ms_ingest * 1e-3), "unit": "rows/s", "ms_per_step": ms_ingest,
                         "rows_per_gpu": NT, "slice_rows": slice_rows, "phases_max_over_ranks": phases,
                         "note": "key-range partitioned table from every rank's unsorted keys: key sample (1024 per "
                                 "rank, gm_key_sample) + splitters (one all_gather), one partition pass "
                                 "(gm_key_partition: count, scan, stable scatter into destination runs), one "
                                 "all-to-all per column (z 8 + bin 2 + 4-B source row = 14 B/row), one sort of the "
                                 "received slice (gm_sort_keys); the slice keeps each row's source beside the sort's "
                                 "permutation (a query maps only its matches); at world 1 the sort is the table"},
        "table_query": {"value": 1.0 / (ms_scan * 1e-3), "unit": "queries/s", "ms_per_step": ms_scan,
                        "table_rows": NT * dist.world, "ranges": nr, "ranges_scanned_rank0": res["ncl"],
                        "rows_scanned": int(scanned), "matches": int(matches), "plan_ms": round(plan_ms, 2),
                        "parity": qparity,
                        "equivalent_scan_rate": NT * dist.world / (ms_scan * 1e-3),
                        "note": "configs[2] query bbox(-10,35,30,60) during 2020-06-01/06-08T12 over the whole "
                                "partitioned table: each rank clips the ranges to its key slice, seeks + Z3Filter, "
                                "maps to global ids, ids gathered to rank 0 (ranges planned once, plan_ms, not in "
                                "ms_per_step)"},
    }


def bench_config0(a, dist, ctx, x, y, t, n0=10_000_000):
    """BASELINE configs[0]: Z3SFC(week) index of 10M points + ranges() for one bbox / time query
    (Z3SFC.scala:37-67, Z3IndexKeySpace.scala:161-194: getIndexValues + getRanges with
    ScanRangesTarget 2000), on the GPU (the key kernel over 10M resident points; the query planned on
    the host and decomposed by gm_z3_ranges through the C ABI) beside the C restatement on the host."""
    import torch
    from geomesa_amd import _lib
    from geomesa_amd.keyspace import Z3IndexKeySpace, during
    lib, h, P = ctx.lib, ctx.handle, _lib.ptr
    n0 = min(n0, x.numel())
    xs, ys, ts = x[:n0], y[:n0], t[:n0]
    b0 = torch.empty(n0, dtype=torch.int16, device=x.device)
    z0 = torch.empty(n0, dtype=torch.int64, device=x.device)

    def idx_step():
        _lib.check(lib.gm_z3_index_key(h, P(xs), P(ys), P(ts), n0, 1, 0, P(b0), P(z0), None, None), "gm_z3_index_key")
    ms_idx = timed(dist, idx_step, 20, 3)
    ks = Z3IndexKeySpace()
    q_box, q_t = (-10.0, 35.0, 30.0, 60.0), (1590969600000, 1591056000000)   # 2020-06-01 during 1 day
    res = {}

    def plan():
        v = ks.get_index_values([q_box], [during(*q_t)])
        res["r"] = ks.get_ranges(v)
        res["v"] = v
    plan()
    reps = 20
    t0 = time.time()
    for _ in range(reps):
        plan()
    ms_rng = (time.time() - t0) * 1e3 / reps
    ms_rng = dist.max(ms_rng)
    out = {"workload": "Z3SFC(week) index of %d points + ranges() of bbox(-10,35,30,60) DURING 2020-06-01/06-02 "
                       "(target 2000)" % n0,
           "gpu": {"index_ms": ms_idx, "index_points_per_s": n0 * dist.world / (ms_idx * 1e-3),
                   "ranges_ms": ms_rng, "ranges": len(res["r"]),
                   "note": "index: the key kernel over resident columns (HIP events); ranges: host planning + "
                           "gm_z3_ranges through the C ABI, wall time per query"}}
    if dist.rank == 0 and not a.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        hx, hy, ht = xs.cpu().numpy(), ys.cpu().numpy(), ts.cpu().numpy()
        t0 = time.time()
        ob, oz, _ = O.z3_index_key_batch(hx, hy, ht)
        cpu_idx = time.time() - t0
        v = res["v"]
        t0 = time.time()
        cpu_r = []
        for bn in sorted(v.temporalBounds):
            cpu_r.append(O.z3_ranges(v.spatialBounds, v.temporalBounds[bn], 64,
                                     max(1, 2000 // len(v.temporalBounds))))
        cpu_rng = time.time() - t0
        # getRanges drops IndexRange.contained (Z3IndexKeySpace.scala:174-194); compare the sfc's own
        # IndexRanges for the same per-bin queries, contained included
        tb = v.temporalBounds
        gpu_ir = ks.sfc.ranges_batch([(v.spatialBounds, tb[bn]) for bn in sorted(tb)], 64, max(1, 2000 // len(tb)))
        gpu_r = [(int(r.lower), int(r.upper), bool(r.contained)) for rr in gpu_ir for r in rr]
        cpu_flat = [(int(r[0]), int(r[1]), bool(r[2])) for rr in cpu_r for r in rr]
        assert len(gpu_r) == len(res["r"])
        # the timed path's own output (getRanges: (bin, lower) / (bin, upper) pairs) against the oracle too
        cpu_bins = [(bn, int(r[0]), int(r[1])) for bn, rr in zip(sorted(tb), cpu_r) for r in rr]
        timed_r = [(int(lo[0]), int(lo[1]), int(hi[1])) for kind, lo, hi in res["r"] if kind == "bounded"]
        out["cpu_baseline"] = {"index_ms": cpu_idx * 1e3, "index_points_per_s": n0 / cpu_idx, "ranges_ms": cpu_rng * 1e3,
                               "cores": 1, "kind": "port", "host": cpu_info(),
                               "sample": "the same %d points and the same query through the C restatement, 1 thread"
                                         % n0}
        out["parity"] = {"keys_equal": bool(np.array_equal(ob, b0.cpu().numpy()) and np.array_equal(oz, z0.cpu().numpy())),
                         "ranges_equal": gpu_r == cpu_flat, "timed_ranges_equal": timed_r == cpu_bins,
                         "ranges": len(cpu_flat),
                         "contained": sum(r[2] for r in cpu_flat),
                         "note": "IndexRange (lower, upper, contained) of every bin's getRanges against the oracle "
                                 "(zorder/sfcurve/package.scala:22-76, ZN.scala:110-242)"}
    del b0, z0
    return out


def all_gather_ints(dist, v):
    if dist.pg is None:
        return [v]
    import torch
    from geomesa_amd.shard import _device_of
    t = torch.tensor([int(v)], dtype=torch.int64, device=_device_of(dist.pg))
    parts = [torch.zeros_like(t) for _ in range(dist.world)]
    dist.pg.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def query_polygon():
    """A deterministic 1,024-vertex query polygon (lobed ring around (10, 47), radius 8-14 deg)
    with a 64-vertex hole: the INTERSECTS geometry of the fused-filter bench lines."""
    from geomesa_amd.join import PolygonSet
    th = np.linspace(0, 2 * np.pi, 1025)[:-1]
    r = 11 + 2.5 * np.sin(5 * th) + 0.5 * np.sin(37 * th)
    ring = [(float(10 + 1.6 * r[i] * np.cos(th[i])), float(47 + r[i] * np.sin(th[i]))) for i in range(len(th))]
    ring.append(ring[0])
    th2 = np.linspace(0, 2 * np.pi, 65)[:-1]
    hole = [(float(12 + 3 * np.cos(a)), float(46 - 2 * np.sin(a))) for a in th2]
    hole.append(hole[0])
    wkt = "POLYGON((%s), (%s))" % (", ".join("%r %r" % p for p in ring), ", ".join("%r %r" % p for p in hole))
    return PolygonSet.from_wkt([wkt])


def _r(v, k=4):
    return None if v is None else (round(v, k) if isinstance(v, float) else v)


def compact(out):
    """The stdout line: the contract fields, the headline roofline / CPU baseline, and the join
    (configs[3], the other half of the metric) with its roofline and parity sample.  Every other leg
    is in the BENCH_DETAIL record (stderr, gpurun_out/bench_detail_n<N>.json)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")
    c = {k: out[k] for k in keep if k in out}
    if "roofline" in out:
        c["roofline"] = {k: _r(out["roofline"].get(k)) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                                 "kernel", "box_copy_gbs", "frac_of_box_copy")}
    cb = out.get("cpu_baseline")
    if cb:
        c["cpu_baseline"] = {"value": _r(cb["value"], 1), "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
                             "threads_1": _r(cb["threads_1"]["value"], 1),
                             "cpu_model": (cb.get("host") or {}).get("cpu_model"),
                             "sample": "oracle, strided sample of this run, 1 and nproc threads",
                             "parity_mismatches": cb["parity_sample"]["mismatches"]}
    pj = out.get("pip_join")
    if pj:
        rf = pj["roofline"]
        j = {"value": _r(pj["value"], 1), "unit": pj["unit"], "ms_per_step": _r(pj["ms_per_step"]),
             "points_per_s": _r(pj["points_per_s"], 1), "matches": pj["matches"],
             "roofline": {"bound": rf["bound"], "achieved": rf["achieved"], "peak": rf["peak"], "unit": rf["unit"],
                          "frac": rf["frac"], "traffic": rf["traffic"],
                          "kernel_fp64_frac": _r((rf.get("fp64") or {}).get("kernel_fp64_frac"), 5),
                          "gather_model_ms": (rf.get("gather_model") or {}).get("model_ms"),
                          "gather_frac": (rf.get("gather_model") or {}).get("frac")}}
        if "row_predicate" in pj:
            j["row_predicate_ms"] = _r(pj["row_predicate"]["ms_per_step"])
        jc = pj.get("cpu_baseline")
        if jc:
            j["cpu_baseline"] = {"value": _r(jc["value"], 1), "cores": jc["cores"], "threads_1": _r(jc["threads_1"]["value"], 1)}
            ps = jc.get("parity_sample")
            if ps:
                j["parity_sample"] = {"points": ps["points"], "pairs": ps["pairs"], "equal": ps["equal"]}
        c["pip_join"] = j
    c["detail"] = "stderr BENCH_DETAIL / gpurun_out/bench_detail_n%d.json" % out.get("n_gpus", 1)
    return c


# ------------------------------------------------------------------------------ main

def main():
    a = parse()
    import torch
    from geomesa_amd import _lib
    from geomesa_amd.curve import Z3SFC, Z2SFC
    dist = Dist(a.gpus)
    ctx = _lib.context(dist.local)
    only = set(a.only.split(",")) if a.only else {"z3", "join", "extra", "table"}
    dev = torch.device("cuda", dist.local)
    N = a.points
    out = {"metric": METRIC, "unit": "points/s", "n_gpus": dist.world, "steps": a.steps, "warmup": a.warmup,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64+int64",
           "data": "synthetic SplitMix64 on device (lon U[-180,180), lat U[-90,90), t U[2020,2021) ms)"}
    extra = {}

    # ---------------------------------------------------------------- Z3 encode (headline)
    x = torch.empty(N, dtype=torch.float64, device=dev)
    y = torch.empty(N, dtype=torch.float64, device=dev)
    t = torch.empty(N, dtype=torch.int64, device=dev)
    b = torch.empty(N, dtype=torch.int16, device=dev)
    z = torch.empty(N, dtype=torch.int64, device=dev)
    lo, _ = shard_bounds(N * dist.world, dist.rank, dist.world)   # this rank's rows of the global set
    gen_points(ctx, N, lo, (-180.0, -90.0, 180.0, 90.0), x, y, t)
    sfc = Z3SFC("week")
    lib, h = ctx.lib, ctx.handle
    P = _lib.ptr

    def z3_step():
        rc = lib.gm_z3_index_key(h, P(x), P(y), P(t), N, 1, 0, P(b), P(z), None, None)
        if rc:
            _lib.check(rc, "gm_z3_index_key")
    ms = None
    if "z3" in only:
        ms = timed(dist, z3_step, a.steps, a.warmup)
        st = _lib.BatchStatus()
        _lib.check(lib.gm_z3_index_key(h, P(x), P(y), P(t), N, 1, 0, P(b), P(z), None, __import__("ctypes").byref(st)),
                   "z3")
        assert st.n_errors == 0
        if dist.rank == 0 and not a.no_cpu:   # strided sample of this run for the CPU leg
            stride = max(1, N // 4_000_000)
            z3_sample = tuple(v[::stride].cpu().numpy() for v in (x, y, t, b, z)) + (stride,)
        total = N * dist.world
        out.update({"value": total / (ms * 1e-3), "ms_per_step": ms})
        out["roofline"] = roofline(34.0 * N, ms, load_pmc("z3_index_key", N))
        out["roofline"]["bytes_per_unit"] = 34
        out["roofline"]["kernel"] = "k_z3_index_key<WEEK,false,false,4>"
        # this box's own streaming ceiling beside the spec peak: the HBM rate of a device-to-device copy
        # of the same 34 GB shape (HBM rates differ between boxes by up to ~15%), so the fraction can be
        # compared across captures
        cp = box_copy_gbs(dist, x, ctx)
        out["roofline"]["box_copy_gbs"] = round(cp, 1)
        out["roofline"]["frac_of_box_copy"] = round(out["roofline"]["achieved"] / cp, 4)
        out["roofline"]["box_copy_note"] = ("4 GB device-to-device copy (gm_device_copy: 16 B per lane, non-temporal, "
                                            "the encode kernels' access shape), best of 6, read + write bytes / time")
    out["config"] = {"workload": "configs[1]: Z3IndexKeySpace.toIndexKey batch (BinnedTime + Z3SFC(week).index), "
                                 "%d resident points per GPU" % N,
                     "points_per_gpu": N, "period": "week", "parallelism": "point shards, no collective"}

    # ---------------------------------------------------------------- extra hot-path kernels on the same data
    if "extra" in only and not a.no_extra:
        def rec(name, fn, bytes_per_unit, n_units, unit="points/s", steps=max(3, a.steps // 2)):
            def step():
                rc = fn()
                if rc:
                    _lib.check(rc, name)
            m = timed(dist, step, steps, 1)
            extra[name] = {"value": n_units * dist.world / (m * 1e-3), "unit": unit, "ms_per_step": m,
                           "roofline": roofline(bytes_per_unit * n_units, m, load_pmc(name, n_units))}
        # the same encode when the caller hands HOST buffers (the JVM boundary without device
        # columns): pinned host -> device copies of 24 B/point, the kernel, 10 B/point back; one
        # 64M-point batch in 8M-point chunks, chunk k+1's H2D and chunk k-1's D2H overlapping chunk
        # k's kernel; checked against the resident-column keys (computed here when the z3 leg is off)
        if "z3" not in only:
            z3_step()
        extra["z3_index_key_host_buffers"] = pcie_encode(dist, ctx, x, y, t, z)
        def elem_parity(name, outs, check):
            """every stride-th element of a full-size encode / decode leg against the oracle (rank 0, untimed)"""
            if dist.rank != 0 or a.no_cpu:
                return
            stride = max(1, N // 2_000_000)
            r = torch.arange(0, N, stride, device=dev, dtype=torch.int64)
            exp = check(r)
            bad = np.zeros(len(r), bool)
            for o, e in zip(outs, exp):
                g = o[r].cpu().numpy()
                bad |= (g.view(np.int64) != np.asarray(e).view(np.int64)) if g.dtype == np.float64 else (g != e)
            extra[name]["parity_sample"] = {"elements": int(len(r)), "stride": stride, "mismatches": int(bad.sum()),
                                            "note": "oracle on every stride-th element (FP64 compared bit for bit)"}
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O   # the checker of the parity samples (untimed, rank 0)
        xi = torch.empty_like(x); yi = torch.empty_like(y); ti = torch.empty_like(t)
        rec("z3_invert", lambda: lib.gm_z3_invert(h, P(z), N, 1, 21, P(xi), P(yi), P(ti)), 32, N)
        elem_parity("z3_invert", (xi, yi, ti), lambda r: O.z3_invert_batch(z[r].cpu().numpy()))
        del xi, yi, ti
        z2 = torch.empty_like(z)
        rec("z2_index", lambda: lib.gm_z2_index(h, P(x), P(y), N, 31, 0, P(z2), None, None), 24, N)
        elem_parity("z2_index", (z2,), lambda r: O.z2_index_batch(x[r].cpu().numpy(), y[r].cpu().numpy())[:1])
        rec("z2_invert", lambda: lib.gm_z2_invert(h, P(z2), N, 31, P(x), P(y)), 24, N)
        elem_parity("z2_invert", (x, y), lambda r: O.z2_invert_batch(z2[r].cpu().numpy()))
        del z2
        # the same encode from a geomesa-arrow-jts PointVector ([y, x] Float8 tuples) + date vector, read in place
        from geomesa_amd.arrow import GeomColumnC, TimeColumnC
        import ctypes
        yx = torch.stack([y, x], 1)
        gcol = GeomColumnC(0, 64, 0, 0, yx.data_ptr(), None, 0, (ctypes.c_void_p * 3)())
        tcol = TimeColumnC(t.data_ptr(), None, 0)
        rec("arrow_z3_keys", lambda: lib.gm_z3_index_key_arrow(h, ctypes.byref(gcol), ctypes.byref(tcol), N, 1, 0, P(b),
                                                              P(z), None, None), 34, N)
        del yx
        # Z3Histogram.observe over the same points (stats caller): 54 week bins of 2020 x 512
        # counters fit the LDS-private path; x 1024 takes the device-atomic path
        hp = torch.zeros(54, dtype=torch.uint8, device=x.device)
        htl = torch.zeros(2, dtype=torch.int64, device=x.device)
        for hl, nm in ((512, "z3_histogram"), (1024, "z3_histogram_1024")):
            hc = torch.zeros((54, hl), dtype=torch.int64, device=x.device)
            rec(nm, lambda: lib.gm_z3_histogram(h, P(x), P(y), P(t), N, 1, hl, 0, 2608, 54, P(hp), P(hc), P(htl)),
                24, N)
            extra[nm]["length"] = hl
            del hc
        # filter scan, key space (configs[2] query on the resident keys)
        from geomesa_amd import filters as F
        from geomesa_amd.keyspace import Z3IndexKeySpace, during
        ks = Z3IndexKeySpace()
        v = ks.get_index_values([(-10, 35, 30, 60)], [during(1590969600000, 1591617600000)])
        fb = F.serialize_to_bytes(F.Z3Filter.from_values(v))
        import ctypes
        fbuf = (ctypes.c_uint8 * len(fb)).from_buffer_copy(fb)
        br = np.asarray(ks.bin_ranges(v), np.int16).reshape(-1)
        mask = torch.empty((N + 63) // 64, dtype=torch.int64, device=dev)
        rec("z3filter_scan", lambda: lib.gm_z3filter_scan(h, fbuf, len(fb), br.ctypes.data, len(br) // 2, P(b), P(z),
                                                         N, P(mask), None, 0, None), 10.125, N, unit="rows/s")
        if dist.rank == 0 and not a.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
        extra["z3filter_scan"]["parity_sample"] = scan_parity(
            dist, a, mask, N, lambda r: O.z3filter_scan(fb, br, b[r].cpu().numpy(), z[r].cpu().numpy()))
        # strict columnar filter (SURVEY 8(d) "Filter scan, strict columnar", 24 B/point): GeoTools BBOX
        # (GeometryProcessing.scala:129) AND FastDuring (FastTemporalOperator.scala:123-126) on x / y / t
        bbq = (ctypes.c_double * 4)(-10.0, 35.0, 30.0, 60.0)
        rec("strict_scan", lambda: lib.gm_strict_scan(h, P(x), P(y), P(t), N, bbq, 1, 1590969600000, 1591617600000,
                                                     P(mask), None, 0, None), 24.125, N, unit="rows/s")
        nm = ctypes.c_int64()
        _lib.check(lib.gm_strict_scan(h, P(x), P(y), P(t), N, bbq, 1, 1590969600000, 1591617600000, P(mask), None, 0,
                                      ctypes.byref(nm)), "strict")
        extra["strict_scan"]["matches"] = nm.value
        extra["strict_scan"]["query"] = "bbox(-10,35,30,60) AND dtg DURING 2020-06-01T00:00Z/2020-06-08T12:00Z"
        extra["strict_scan"]["parity_sample"] = scan_parity(
            dist, a, mask, N, lambda r: O.strict_scan(x[r].cpu().numpy(), y[r].cpu().numpy(), t[r].cpu().numpy(),
                                                      (-10.0, 35.0, 30.0, 60.0), (1590969600000, 1591617600000)))
        # fused full filter (north star: bbox + time window + point-in-polygon in one pass) over the
        # resident x/y/t columns: a 1,024-vertex query polygon with a hole around Europe, as
        # (a) INTERSECTS + BBOX + DURING (the Z3 query of the filter scan above) and (b) INTERSECTS alone
        from geomesa_amd.join import PolygonIndex, PolygonSet
        qpoly = query_polygon()
        qix = PolygonIndex(qpoly, cells_per_poly=65536)
        qmask = torch.empty((N + 63) // 64, dtype=torch.int64, device=dev)
        rec("query_scan", lambda: lib.gm_query_scan(h, P(x), P(y), P(t), N, bbq, 1, 1590969600000, 1591617600000, qix._h,
                                                   1, P(qmask), None, 0, None), 24.125, N, unit="rows/s")
        qoracle = O.OraclePolySet(*qpoly.to_arrays()) if dist.rank == 0 and not a.no_cpu else None
        extra["query_scan"]["parity_sample"] = scan_parity(
            dist, a, qmask, N, lambda r: O.query_scan(x[r].cpu().numpy(), y[r].cpu().numpy(), t[r].cpu().numpy(),
                                                      (-10.0, 35.0, 30.0, 60.0), (1590969600000, 1591617600000),
                                                      polys=qoracle, op=1))
        rec("query_scan_polygon", lambda: lib.gm_query_scan(h, P(x), P(y), None, N, None, 0, 0, 0, qix._h, 1, P(qmask),
                                                           None, 0, None), 16.125, N, unit="rows/s")
        extra["query_scan_polygon"]["parity_sample"] = scan_parity(
            dist, a, qmask, N, lambda r: O.query_scan(x[r].cpu().numpy(), y[r].cpu().numpy(), polys=qoracle, op=1))
        nm = ctypes.c_int64()
        _lib.check(lib.gm_query_scan(h, P(x), P(y), None, N, None, 0, 0, 0, qix._h, 1, P(qmask), None, 0,
                                     ctypes.byref(nm)), "query")
        extra["query_scan_polygon"]["matches"] = nm.value
        extra["query_scan_polygon"]["polygon"] = "1,024-vertex ring + 64-vertex hole, envelope 40 x 24 deg; 65,536-cell index"
        del qmask, qix
        del mask
        # XZ2 / XZ3 index of 100M envelopes (configs[4]): x/y as min corners, max corners a log-uniform
        # [1e-6, 10] deg away; XZ3 time extent 1 s .. 1 day inside the week
        NX = min(N, 100_000_000)
        g = torch.Generator(device=dev).manual_seed(11)
        w = torch.pow(10.0, torch.rand(NX, device=dev, dtype=torch.float64, generator=g) * 7 - 6)
        hgt = torch.pow(10.0, torch.rand(NX, device=dev, dtype=torch.float64, generator=g) * 7 - 6)
        xmax = torch.clamp(x[:NX] + w, max=180.0); ymax = torch.clamp(y[:NX] + hgt, max=90.0)
        del w, hgt
        xo = torch.empty(NX, dtype=torch.int64, device=dev)
        rec("xz2_index", lambda: lib.gm_xz2_index(h, P(x), P(y), P(xmax), P(ymax), NX, 12, 0, P(xo), None, None), 40,
            NX, unit="envelopes/s")
        xstride = max(1, NX // 1_000_000)

        def xz_parity(name, cols, fn):
            """every xstride-th envelope of the full-size run keyed by the oracle (XZ2SFC.scala:54-77,
            XZ3SFC.scala:53-76) against the keys the GPU wrote"""
            if dist.rank != 0 or a.no_cpu:
                return
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            env = np.stack([c[:NX:xstride].cpu().numpy() for c in cols], 1)
            ok, ost = getattr(O, fn)(env)
            gk = xo[:NX:xstride].cpu().numpy()
            extra[name]["parity_sample"] = {"envelopes": len(env), "stride": xstride,
                                            "mismatches": int(((ok != gk) | (ost != 0)).sum())}
        xz_parity("xz2_index", (x, y, xmax, ymax), "xz2_index_batch")
        zmin = torch.remainder(t[:NX], 604_800_000).to(torch.float64) / 1000.0
        zmax = torch.clamp(zmin + torch.pow(10.0, torch.rand(NX, device=dev, dtype=torch.float64, generator=g) * 4.94),
                           max=604800.0)
        rec("xz3_index", lambda: lib.gm_xz3_index(h, P(x), P(y), P(zmin), P(xmax), P(ymax), P(zmax), NX, 12, 1, 0, P(xo),
                                                 None, None), 56, NX, unit="envelopes/s")
        xz_parity("xz3_index", (x, y, zmin, xmax, ymax, zmax), "xz3_index_batch")
        del xmax, ymax, xo, zmin, zmax
        # batched ranges (configs[4]): the queries sharded over the ranks (contiguous blocks), every
        # rank decomposes its block, offsets + ranges gathered to rank 0 (shard.gather_ranges)
        from geomesa_amd import ranges as R
        rng = np.random.default_rng(2)
        nq = 100_000
        wq = 10 ** rng.uniform(-2, np.log10(20), (nq, 2)) / 2
        cq = np.stack([rng.uniform(-180 + wq[:, 0], 180 - wq[:, 0]), rng.uniform(-90 + wq[:, 1], 90 - wq[:, 1])], 1)
        win = np.ascontiguousarray(np.concatenate([cq - wq, cq + wq], 1))
        tw0 = rng.uniform(0, 604800 - 172800, nq)
        tw1 = tw0 + 10 ** rng.uniform(np.log10(60), np.log10(172800), nq)
        win3 = np.ascontiguousarray(np.stack([win[:, 0], win[:, 1], tw0, win[:, 2], win[:, 3], tw1], 1))
        qlo, qhi = shard_bounds(nq, dist.rank, dist.world)
        wl, wl3 = np.ascontiguousarray(win[qlo:qhi]), np.ascontiguousarray(win3[qlo:qhi])
        woff = np.arange(qhi - qlo + 1, dtype=np.int32)
        note = ("C-ABI call incl. H2D of the windows and D2H of the ranges (pinned host output: query chunks "
                "pipelined with their result copies), queries "
                "sharded over the ranks with offsets + ranges gathered to rank 0; 100k %s query windows "
                "(0.01-20 deg%s), maxRanges 2000, g = 12")
        m, gl = ranges_batch(dist, lib.gm_xz2_ranges, (h, qhi - qlo, woff.ctypes.data, wl.ctypes.data, 12, 2000),
                             qhi - qlo, nq)
        extra["xz2_ranges_batch"] = dict(m, note=note % ("XZ2", ""))
        if dist.rank == 0 and not a.no_cpu:
            extra["xz2_ranges_batch"].update(cpu_ranges_baseline("xz2", win, None, 2000, m["ms_per_step"], nq, gl, m.get("device_output", {}).get("ms_per_step")))
        del gl
        m, gl = ranges_batch(dist, lib.gm_xz3_ranges, (h, qhi - qlo, woff.ctypes.data, wl3.ctypes.data, 12, 1, 2000),
                             qhi - qlo, nq)
        extra["xz3_ranges_batch"] = dict(m, note=note % ("XZ3", " x 1 min-2 days, week period"))
        if dist.rank == 0 and not a.no_cpu:
            extra["xz3_ranges_batch"].update(cpu_ranges_baseline("xz3", win3, None, 2000, m["ms_per_step"], nq, gl, m.get("device_output", {}).get("ms_per_step")))
        del gl
        # batched Z3 ranges (configs[4]/[0]): 4096 queries with target 2000
        rng = np.random.default_rng(1)
        qs = []
        for _ in range(4096):
            w = 10 ** rng.uniform(-1, 1); hh = 10 ** rng.uniform(-1, 1)
            cx = rng.uniform(-170, 170); cy = rng.uniform(-80, 80); t0 = int(rng.integers(0, 500000))
            qs.append(([(cx - w, cy - hh, cx + w, cy + hh)], [(t0, t0 + 86400)]))
        qlo, qhi = shard_bounds(len(qs), dist.rank, dist.world)
        fn, args, n3, _ = R.prepare_z3(sfc, qs[qlo:qhi], 64, 2000)
        m, gl = ranges_batch(dist, fn, args, n3, len(qs))
        extra["z3_ranges_batch"] = dict(m, note="C-ABI call incl. H2D of queries and D2H of ranges (pinned host "
                                                "output), sharded over the ranks + gather to rank 0; 4096 Z3 queries "
                                                "(0.2-20 deg boxes x 1 day), maxRanges 2000 (ScanRangesTarget)")
        if dist.rank == 0 and not a.no_cpu:
            qb = np.array([q[0][0] for q in qs], np.float64)
            qt = np.array([q[1][0] for q in qs], np.int64)
            extra["z3_ranges_batch"].update(cpu_ranges_baseline("z3", qb, qt, 2000, m["ms_per_step"], len(qs), gl, m.get("device_output", {}).get("ms_per_step")))
        del gl
    # ---------------------------------------------------------------- configs[0]: 10M-point index + one query's ranges
    if "extra" in only and not a.no_extra:
        extra["config0"] = bench_config0(a, dist, ctx, x, y, t)
    # ---------------------------------------------------------------- sorted table: ingest sort + seek-and-filter
    if "table" in only and not a.no_extra:
        try:   # a failure here (every rank alike, e.g. a collective the backend refuses) keeps the line
            extra.update(bench_table(a, dist, ctx, b, z))
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            extra["table_error"] = repr(e)[:300]
            torch.cuda.synchronize()
    del x, y, t, b, z
    torch.cuda.empty_cache()

    # ---------------------------------------------------------------- st_contains join (configs[3])
    if "join" in only:
        from geomesa_amd.join import PolygonIndex, PolygonSet, synthetic_counties
        J = a.join_points
        gx, gy = (int(v) for v in a.join_grid.split("x"))
        ps = synthetic_counties(gx, gy) if dist.rank == 0 else None
        # rank 0 builds the index; with more ranks its device arrays are broadcast over RCCL (the
        # reference ships the polygon side with the Spark join shuffle) and imported, no rebuild
        dist.barrier()
        t_ix = time.time()
        ix = PolygonIndex(ps, ctx, a.cells_per_poly) if dist.rank == 0 else None
        t_build = time.time() - t_ix
        if dist.pg is not None:
            from geomesa_amd.shard import broadcast_index
            ix = broadcast_index(dist.pg, ix, 0, ctx)
        torch.cuda.synchronize()
        t_ix = dist.max(time.time() - t_ix)
        t_build = dist.max(t_build if dist.rank == 0 else 0.0)
        n_polys = int(dist.max(ps.n_polys if ps is not None else 0))
        n_verts = int(dist.max(ps.n_vertices if ps is not None else 0))
        px = torch.empty(J, dtype=torch.float64, device=dev)
        py = torch.empty(J, dtype=torch.float64, device=dev)
        jlo, _ = shard_bounds(J * dist.world, dist.rank, dist.world)
        gen_points(ctx, J, jlo + (1 << 40), CONUS, px, py, None)
        if a.join_sorted:   # locality experiment only (not a bench configuration)
            py, order = torch.sort(py)
            px = px[order]
            del order
        jmode = PolygonIndex.MODES[a.join_mode]
        cnt = ix.join(px, py, count_only=True, mode=a.join_mode)
        cap = int(cnt * 1.05) + 1024
        ptids = torch.empty(cap, dtype=torch.int64, device=dev)
        plids = torch.empty(cap, dtype=torch.int32, device=dev)
        npairs = __import__("ctypes").c_int64()

        def join_step():
            rc = lib.gm_pip_join_ex(h, ix._h, P(px), P(py), J, jlo, P(ptids), P(plids), cap, None, jmode)
            if rc:
                _lib.check(rc, "gm_pip_join")
        jms = timed(dist, join_step, a.join_steps, 1)
        _lib.check(lib.gm_pip_join_ex(h, ix._h, P(px), P(py), J, jlo, P(ptids), P(plids), cap,
                                      __import__("ctypes").byref(npairs), jmode), "join")
        matches = int(dist.sum(npairs.value))
        census = ix.census(px, py)   # how the lookup chain resolves these points (diagnostic, untimed)
        pairs = J * n_polys * dist.world
        pj = {"value": pairs / (jms * 1e-3), "unit": "pairs/s",
              "points_per_s": J * dist.world / (jms * 1e-3), "matches_per_s": matches / (jms * 1e-3),
              "value_note": "value = logical (point, polygon) pairs resolved per second, N_points x N_polygons / t "
                            "(SURVEY 8(d)); the work-based rates are points_per_s and matches_per_s",
              "ms_per_step": jms, "points_per_gpu": J,
              "polygons": n_polys, "vertices": n_verts, "matches": matches,
              "index_build_s": round(t_build, 3), "index_ready_s": round(t_ix, 3), "index": ix.stats(), "mode": a.join_mode,
              "census": census,
              "roofline": roofline(16.0 * J + 12.0 * npairs.value, jms, load_pmc("pip_join", J)),
              "workload": "st_contains(polygon, point) join, %d CONUS points/GPU x %d synthetic county polygons "
                          "(BASELINE configs[3]); index built on rank 0, broadcast over RCCL when N > 1"
                          % (J, n_polys)}
        pj["roofline"]["bytes_per_unit"] = "16 B/point + 12 B/pair"
        pj["roofline"]["gather_model"] = gather_model(census, J, npairs.value, jms)
        tr = pj["roofline"].get("traffic")
        if tr:   # the calibrated view: every L2 miss moves a whole 128-B line (tools/traffic_probe.hip), so the
            # kernel's own line traffic (PMC bytes) against the box's streaming rate is its bandwidth roofline
            pj["roofline"]["line_traffic"] = {
                "bytes": tr, "over_algorithmic": round(tr / (16.0 * J + 12.0 * npairs.value), 3),
                "gbs": round(tr / (jms * 1e-3) / 1e9, 1), "stream_gbs": PROBE_STREAM_GBS,
                "frac_of_stream": round(tr / (jms * 1e-3) / 1e9 / PROBE_STREAM_GBS, 4),
                "note": "PMC read bytes = 128 B per memory-side read request (TCC_EA0_RDREQ_128B) + WRITE_SIZE, from "
                        "profiles/pmc_traffic.json; the join is bound by these whole-line misses"}
        # FP64 work: E_c = the edges of every (point, polygon) pair whose envelope test
        # passes, counted by the C restatement over a prefix of the same device point stream, scaled;
        # 7 FP64 ops per candidate edge is the reference walk's orientation arithmetic
        if dist.rank == 0 and not a.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            ns = min(J, 20_000_000)
            _, _, ec = O.OraclePolySet(*ps.to_arrays()).join(px[:ns].cpu().numpy(), py[:ns].cpu().numpy(),
                                                            nthreads=cpu_threads(), with_edges=True)
            ec_total = ec * (J / ns)
            fl = 7.0 * ec_total * dist.world
            pj["roofline"]["fp64"] = {"e_c_per_point": ec / ns, "e_c": ec_total, "flops": fl,
                                      "reference_equivalent_tflops": fl / (jms * 1e-3) / 1e12, "peak_tflops": FP64_PEAK_TFLOPS,
                                      "reference_equivalent_fp64": fl / (jms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                                      "sample": "E_c counted by the oracle over the first %d of the %d points, scaled" % (ns, J),
                                      "note": "NOT a roofline fraction: the reference's per-pair RayCrossingCounter work "
                                              "(7 FP64 ops x E_c) over the GPU's time -- work the grid index avoids; the "
                                              "kernel's own FP64 roofline is kernel_fp64_frac"}
            fpm = load_profile("pip_join_fp64", J)
            if fpm:   # what the kernel itself executes: SQ_INSTS_VALU_FLOPS_FP64 (FLOPs per wave
                # instruction, gfx950) x 64 lanes, an upper bound (inactive lanes counted)
                kf = 64.0 * fpm["sq_insts_valu_flops_fp64"] * dist.world
                pj["roofline"]["fp64"].update(
                    sq_insts_valu_flops_fp64=fpm["sq_insts_valu_flops_fp64"], kernel_flops_max=kf,
                    kernel_fp64_frac=kf / (jms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                    kernel_note="profiles/pmc_traffic.json pip_join_fp64: the grid kernel's own FP64 work is "
                                "far below the FP64 peak; the join is bound by dependent index loads")
        # row-wise st_contains (the UDF path without the join rule): row i = (its cell's county, point i)
        x0c, y0c, x1c, y1c = CONUS
        rid = (torch.clamp(((py - y0c) / (y1c - y0c) * gy).long(), 0, gy - 1) * gx +
               torch.clamp(((px - x0c) / (x1c - x0c) * gx).long(), 0, gx - 1)).to(torch.int32)
        loc = torch.empty(J, dtype=torch.uint8, device=dev)

        def relate_step():
            rc = lib.gm_pip_relate(h, ix._h, P(rid), P(px), P(py), J, P(loc))
            if rc:
                _lib.check(rc, "gm_pip_relate")
        rms = timed(dist, relate_step, max(3, a.join_steps), 1)
        rp = load_profile("pip_relate", J)
        pj["row_predicate"] = {"value": J * dist.world / (rms * 1e-3), "unit": "rows/s", "ms_per_step": rms,
                               "contains": int(dist.sum(int((loc == 2).sum()))),
                               "roofline": roofline(21.0 * J, rms, rp["bytes_per_launch"] if rp else None),
                               "workload": "st_contains(polygon_i, point_i) row by row over the join's points, "
                                           "polygon_i = the county of the point's grid cell (21 B/row: 16 point + 4 id + 1 out)"}
        del rid, loc

        join_sample = None
        if dist.rank == 0 and not a.no_cpu:   # every stride-th point of this run and the GPU's pairs for them
            stride = max(1, J // 2_000_000)
            npv = int(npairs.value)
            sel = ((ptids[:npv] - jlo) % stride) == 0
            join_sample = (px[::stride].cpu().numpy(), py[::stride].cpu().numpy(), stride,
                           torch.stack([(ptids[:npv][sel] - jlo) // stride, plids[:npv][sel].to(torch.int64)], 1).cpu().numpy())
            del sel
        del px, py
        torch.cuda.empty_cache()
        if not a.no_gather:
            pj["gather"] = gather_pairs(dist, ptids, plids, int(npairs.value), jlo, n_polys)
        if dist.rank == 0 and not a.no_cpu:
            pj["cpu_baseline"] = cpu_join_baseline(a.cpu_seconds, ps, join_sample)
        out["pip_join"] = pj
        del ptids, plids, ix

    if dist.rank == 0 and not a.no_cpu and "z3" in only:
        out["cpu_baseline"] = cpu_z3_baseline(a.cpu_seconds, z3_sample)
    if extra:
        out["extra"] = extra
    if dist.rank == 0:
        # the full record (every leg) goes to stderr and a file; stdout gets ONE compact line that
        # fits the driver's 2,000-character tail with the join's numbers in it
        detail = json.dumps(out)
        print("BENCH_DETAIL " + detail, file=sys.stderr, flush=True)
        try:
            os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
            with open(os.path.join(ROOT, "gpurun_out", "bench_detail_n%d.json" % dist.world), "w") as f:
                f.write(detail + "\n")
        except OSError:
            pass
        print(json.dumps(compact(out)), flush=True)
    if dist.pg:
        dist.pg.destroy_process_group()


if __name__ == "__main__":
    main()
