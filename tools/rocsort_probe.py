"""Times torch.sort (rocPRIM onesweep radix sort) on 250M int64 keys, as a yardstick for the digit pass
of gm_sort_keys: run under rocprofv3 --kernel-trace --stats to see its passes and their times.

    python tools/rocsort_probe.py [rows]
"""
import sys

import torch


def main(n=250_000_000):
    g = torch.Generator(device="cuda").manual_seed(5)
    cases = {
        "u64_random": torch.randint(-2**63, 2**63 - 1, (n,), device="cuda", generator=g, dtype=torch.int64),
        "28bit": torch.randint(0, 2**28, (n,), device="cuda", generator=g, dtype=torch.int64),
    }
    for name, k in cases.items():
        for stable in (False, True):
            torch.sort(k, stable=stable)
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                torch.sort(k, stable=stable)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            print("%s stable=%s: %d rows, best %.2f ms" % (name, stable, n, min(ts)), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 250_000_000)
