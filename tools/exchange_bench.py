"""Times the survivor exchange's pieces at world 1 (GPU): cdx_pack_survivors, the header read, the
whole bench.py exchange — host wall time per call, median of 50.

  python tools/exchange_bench.py [--E 4096]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from compliancedex_amd import distributed as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--E", type=int, default=4096)
    a = ap.parse_args()
    E, T, Dd = a.E, 4, 16
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    f64 = dict(dtype=torch.float64, device=dev)
    margin = torch.rand(E, T, generator=g, **f64) - 0.3
    loss, q, comp = torch.rand(E, generator=g, **f64), torch.rand(E, Dd, generator=g, **f64), torch.rand(E, T, generator=g, **f64)
    target, palm = torch.rand(E, T, 3, generator=g, **f64), torch.rand(E, 6, generator=g, **f64)

    def timed(fn, n=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts) * 1e3

    pack = timed(lambda: D.pack_survivors(E, 0, 0, 0, loss, margin, q, comp, target, palm))
    buf = D.pack_survivors(E, 0, 0, 0, loss, margin, q, comp, target, palm)
    unpack = timed(lambda: D.unpack_records([buf]))
    whole = timed(lambda: D.unpack_records([D.pack_survivors(E, 0, 0, 0, loss, margin, q, comp, target, palm)]))
    sync = timed(lambda: None)
    print(json.dumps({"E": E, "pack_ms": pack, "unpack_ms": unpack, "pack_unpack_ms": whole, "empty_sync_ms": sync}))


if __name__ == "__main__":
    main()
