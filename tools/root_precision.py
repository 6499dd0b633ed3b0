"""Precision of a library build's GPIS mean / std against the oracle (the f32-seeded-root A/Bs).

  CDX_LIB=... python tools/root_precision.py TAG

On the synthetic 2000-point state (cond(E11) ≈ 1e7) and the stored banana state: mean, ∇mean, std at
20 000 random points around the object on the device, the oracle (the reference's algorithm in f64
torch on the CPU) at 200 of them.  Prints one JSON line with max relative errors (max|a − b| / max|b|)
and saves the device outputs to gpurun_out/prec_TAG.npz for cross-build comparison.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from compliancedex_amd.workloads import stored_gpis, synthetic_banana_gpis  # noqa: E402
from tests._helpers import oracle_gpis, oracle_gpis_at, rel_err  # noqa: E402


def main(tag):
    out, rec = {}, {"tag": tag, "lib": os.environ.get("CDX_LIB", "libcdx.so")}
    for state in ("synthetic2000", "banana"):
        g = synthetic_banana_gpis(2000, "cuda") if state == "synthetic2000" else stored_gpis(state, "cuda")
        rng = np.random.default_rng(7)
        X1 = g.X1.cpu().numpy()
        lo, hi = X1.min(0) - 0.02, X1.max(0) + 0.02
        X = lo + (hi - lo) * rng.random((20000, 3))
        Xt = torch.from_numpy(X).cuda().requires_grad_(True)
        mean, std = g.pred(Xt)
        gm, = torch.autograd.grad(mean.sum(), Xt)
        mean, std, gm = mean.detach().cpu().numpy(), std.detach().cpu().numpy(), gm.cpu().numpy()
        idx = rng.choice(len(X), 200, replace=False)
        ref = oracle_gpis_at(oracle_gpis(state), X[idx], with_std=True)
        rec[state] = {"mean": rel_err(mean[idx], ref["mean"]), "gmean": rel_err(gm[idx], ref["gmean"]),
                      "std": rel_err(std[idx], ref["std"])}
        out.update({f"{state}_mean": mean, f"{state}_gmean": gm, f"{state}_std": std})
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez(f"gpurun_out/prec_{tag}.npz", **out)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
