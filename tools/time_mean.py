"""Times cdx_gpis_mean (mean + ∇mean at M queries, synthetic banana GPIS of N points).

  python tools/time_mean.py [M] [N] [reps]

Used alone (HIP events) and under rocprofv3 --pmc to read the mean kernel's VALU issue counters.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(M=16384, N=2000, reps=50):
    import numpy as np
    import torch
    from compliancedex_amd.gpis import gpis_mean
    from compliancedex_amd.workloads import synthetic_banana_gpis
    g = synthetic_banana_gpis(N, "cuda")
    st = g.native_state()
    X1 = g.X1.cpu().numpy()
    rng = np.random.default_rng(0)
    lo, hi = X1.min(0) - 0.03, X1.max(0) + 0.03
    X = torch.from_numpy(lo + (hi - lo) * rng.random((M, 3))).cuda()
    for _ in range(3):
        gpis_mean(st, X)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        mean, gm, _ = gpis_mean(st, X)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    print(json.dumps({"M": M, "N": N, "ms": ms, "pairs_per_s": M * N / (ms * 1e-3),
                      "mean_checksum": float(mean.double().sum())}))
    # the same launches interleaved with the whitened std pass (as inside the closure): the mean
    # kernel's own events, the GPU otherwise busy with fp64 MFMA work
    from compliancedex_amd.gpis import gpis_std
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in evs:
        gpis_std(st, X, want_grad=False)
        e0.record()
        gpis_mean(st, X)
        e1.record()
    torch.cuda.synchronize()
    ms_busy = sum(e0.elapsed_time(e1) for e0, e1 in evs) / reps
    print(json.dumps({"M": M, "N": N, "ms_between_std_passes": ms_busy}))


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:]]
    main(*a)
