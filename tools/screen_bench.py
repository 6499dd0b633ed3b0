"""GPU check of the split-precision variance screen (cdx_gpis_screen_var) on the bench workload:
error vs the fp64 whitened pass (cdx_gpis_std) and kernel times of both.

  python tools/screen_bench.py [--E 4096] [--reps 20]   (writes one JSON line)
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def alltip_queries(E, seed=1000):
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs
    from oracle.cdx_oracle import OracleChain, OracleProblem
    cfg = load_robot("allegro")["config"]
    prob = OracleProblem(OracleChain(load_robot("allegro")["bodies"]), cfg["ee_link_name"], cfg["ee_link_offset"],
                         cfg["ref_q"], None)
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=seed, spread=True)
    with torch.no_grad():
        pre = prob.forward_kinematics(torch.from_numpy(q), torch.from_numpy(palm)).double()
    tgt = torch.from_numpy(target)
    return (tgt + 0.8 * (pre - tgt)).reshape(-1, 3)


def timed(fn, reps):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--E", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from compliancedex_amd.gpis import gpis_std
    from compliancedex_amd.workloads import synthetic_banana_gpis
    g = synthetic_banana_gpis(2000, device="cuda")
    st = g.native_state()
    X = alltip_queries(a.E).cuda()
    k0 = float(g.R) ** 3
    sv = st.screen_var(X)
    std, _ = gpis_std(st, X, want_grad=False)
    torch.cuda.synchronize()
    s2 = std.double() ** 2
    err = ((sv.abs() - s2).abs() / k0).cpu().numpy()
    ex = s2.view(-1, 4).cpu().numpy()
    es = sv.view(-1, 4).cpu().numpy()
    amax = ex.argmax(1)
    out = {"E": a.E, "M": int(X.shape[0]), "err_max_over_k0": float(err.max()),
           "err_p99_over_k0": float(np.percentile(err, 99)), "finite": bool(np.isfinite(es).all())}
    for mult in (8, 32):
        d = mult * err.max() * k0
        cand = (es + d) >= (es - d).max(1, keepdims=True)
        out[f"tips_kept_{mult}x"] = float(cand.sum(1).mean())
        out[f"argmax_kept_{mult}x"] = bool(cand[np.arange(len(amax)), amax].all())
    out["screen_ms"] = timed(lambda: st.screen_var(X), a.reps)
    out["std_fp64_ms"] = timed(lambda: gpis_std(st, X, want_grad=False), a.reps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
