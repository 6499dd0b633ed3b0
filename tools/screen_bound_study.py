"""Can the screen's selection margin be a rigorous a-priori bound?  (CPU study, config 2 rows.)

For the synthetic N = 2000 banana state and the bench's all-tip rows it prints
  * the spectrum facts a norm-wise bound needs: λ_min/λ_max of E11, ‖L⁻¹‖₂, ‖L⁻¹‖_F;
  * the rigorous per-row bounds of the estimate's error terms (operand representation, exact
    products, fp32 accumulation) in units of k0;
  * how many fingertips per (candidate) group the selection would keep at a margin of Δ·k0 for
    Δ from the calibrated 1.6e-4 up to the rigorous bounds (exact std² used as the estimate).

  PYTHONPATH=. python tools/screen_bound_study.py [--E 1024]
"""
import argparse

import numpy as np
import scipy.linalg as sl
import torch

from compliancedex_amd.urdf import load_robot
from compliancedex_amd.workloads import prob_inputs, synthetic_banana_arrays
from oracle.cdx_oracle import OracleChain, OracleGPIS, OracleProblem


def kept_per_group(s2, delta_rows):
    """Selection of cdx_screen.hip screen_select_kernel on a = |s2| with per-row margins."""
    a = np.abs(s2).reshape(-1, 4)
    d = delta_rows.reshape(-1, 4)
    lo = (a - d).max(1, keepdims=True)
    keep = (a + d) >= lo
    return keep.sum(1).mean(), (keep.sum(1) == 4).mean()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--E", type=int, default=1024)
    a = ap.parse_args()
    cfg = load_robot("allegro")["config"]
    X1, y, noise = synthetic_banana_arrays(2000)
    g = OracleGPIS.fit(X1, y, noise, bias=1.0)
    prob = OracleProblem(OracleChain(load_robot("allegro")["bodies"]), cfg["ee_link_name"], cfg["ee_link_offset"],
                         cfg["ref_q"], g)
    q, comp, target, palm = prob_inputs(cfg["ref_q"], a.E, seed=1000, spread=True)
    with torch.no_grad():
        pre = prob.forward_kinematics(torch.from_numpy(q), torch.from_numpy(palm)).double()
    tgt = torch.from_numpy(target)
    tips = (tgt + 0.8 * (pre - tgt)).reshape(-1, 3).numpy()
    E11 = g.E11.numpy()
    N = len(E11)
    lam = np.linalg.eigvalsh(E11)
    L = np.linalg.cholesky(E11)
    Li = sl.solve_triangular(L, np.eye(N), lower=True)
    R = float(g.R)
    k0 = R ** 3
    X1d = g.X1.numpy()
    d = tips[:, None, :] - X1d[None, :, :]
    r = np.sqrt((d * d).sum(-1))
    K = 2 * r ** 3 - 3 * R * r ** 2 + R ** 3
    V = K @ Li.T
    s2 = k0 - (V * V).sum(1)
    Lin2 = 1.0 / np.sqrt(lam[0])
    LinF = np.sqrt((Li * Li).sum())
    print(f"N={N} k0=R³={k0:.4g}  λ_min={lam[0]:.3e} λ_max={lam[-1]:.3e} cond={lam[-1] / lam[0]:.3e}")
    print(f"‖L⁻¹‖₂·√k0 = {Lin2 * np.sqrt(k0):.3e}   ‖L⁻¹‖_F·√k0 = {LinF * np.sqrt(k0):.3e}")
    Vn = np.sqrt((V * V).sum(1))
    print(f"‖V‖/√k0: median {np.median(Vn) / np.sqrt(k0):.3f} max {Vn.max() / np.sqrt(k0):.3f}")
    A = K - k0
    An = np.sqrt((A * A).sum(1))
    u = 2.0 ** -24
    # (1) fp32 generation of Ã (centred fp32 coordinates, fp32 r, polynomial): per entry ≤ c·u·(terms),
    #     terms = 2r³ + 3Rr² + |k'(r)|·(|q − c| + |x_n − c|) with c ≈ 8 (a generous count of roundings)
    ctr = X1d.mean(0)
    qn = np.linalg.norm(tips - ctr, axis=1)[:, None]
    xn = np.linalg.norm(X1d - ctr, axis=1)[None, :]
    dA = 8 * u * (2 * r ** 3 + 3 * R * r ** 2 + np.abs(6 * r * (r - R)) * (qn + xn))
    gen = np.sqrt((dA * dA).sum(1)) * Lin2  # ‖δÃ‖₂ ‖L⁻ᵀ‖₂ ≥ ‖δÃ·L⁻ᵀ‖₂
    # (2) split of Ã to 2 fp16 slices (truncation): |δ| ≤ 2⁻²⁰|Ã| (+ fp16 subnormal floor, ignored)
    spl = 2.0 ** -20 * An * Lin2
    # (3) fp32 accumulation of the 3·K slice products (16 per MFMA, one rounding per chunk): per output
    #     ≤ γ·Σ_n |Ã_n||L⁻ᵀ_nj|,  γ = (3·K/16)·u
    gam = 3 * (N / 16) * u
    acc_col = gam * (np.abs(A) @ np.abs(Li.T))  # [M, N]
    acc = np.sqrt((acc_col * acc_col).sum(1))
    for name, e in (("fp32 generation", gen), ("fp16 split of Ã", spl), ("fp32 accumulation", acc)):
        b = 2 * Vn * e + e * e  # |Σ Ṽ² − Σ V²| ≤ 2‖V‖‖δV‖ + ‖δV‖²
        print(f"rigorous bound on |Δstd²|/k0 from {name:18s}: median {np.median(b) / k0:.3e} max {b.max() / k0:.3e}")
    tot = gen + spl + acc
    btot = 2 * Vn * tot + tot * tot
    print(f"sum of bounds: median {np.median(btot) / k0:.3e}")
    print("kept fingertips per group (of 4) at margin Δ·k0 on every row, and the share of groups keeping all 4:")
    for dl in (1.6e-4, 1e-3, 1e-2, 1e-1, 1.0):
        m, full = kept_per_group(s2, np.full(s2.shape, dl * k0))
        print(f"  Δ = {dl:.1e}: {m:.3f} per group, {100 * full:.1f} % of groups keep all 4")
    m, full = kept_per_group(s2, btot)
    print(f"  per-row rigorous bounds: {m:.3f} per group, {100 * full:.1f} % keep all 4")


if __name__ == "__main__":
    main()
