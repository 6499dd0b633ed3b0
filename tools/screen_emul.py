"""Bit-level emulation of the split-precision screen GEMM (CPU only): Ṽ = K*·L⁻ᵀ with both operands
split into slices, the slice products accumulated into ONE fp32 accumulator per output, 16 K at a
time as v_mfma_f32_32x32x16_{bf16,f16} does (the 16 products of a K-chunk summed exactly, one fp32
rounding per chunk add).  bf16 variants (the first version: x ≈ x0 + x1 + x2, six products of
slice-index sum ≤ 2): K* computed in f64 and rounded (ref), K* from fp32 arithmetic on f64
differences, and the R³-offset form (A = K* − R³, V = A·L⁻ᵀ + R³·colsum(L⁻ᵀ)).  fp16 variant (the
kernel now): A·SA and L⁻ᵀ·SB_j (powers of two) split into two fp16 slices — A truncated as
v_cvt_pkrtz_f16_f32 does, L⁻ᵀ rounded to nearest — three products of index sum ≤ 1.  Prints the
std² error / k0 and the ambiguity the screen leaves at margins of 4× / 8× / 16× the max error.

  PYTHONPATH=. python tools/screen_emul.py [--E 1024]
"""
import argparse

import numpy as np
import scipy.linalg as sl
import torch

from compliancedex_amd.urdf import load_robot
from compliancedex_amd.workloads import prob_inputs, synthetic_banana_arrays
from oracle.cdx_oracle import OracleChain, OracleGPIS, OracleProblem


def bf16(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).bfloat16().double().numpy()


def split3(x):
    x = np.asarray(x, dtype=np.float32).astype(np.float64)  # operands reach the splitter as fp32
    a = bf16(x)
    b = bf16(x - a)
    c = bf16(x - a - b)
    return [a, b, c]


def f16(x):
    return np.asarray(x, dtype=np.float32).astype(np.float16).astype(np.float64)


def f16rtz(x):
    x = np.asarray(x, dtype=np.float32)
    h = x.astype(np.float16)
    over = np.abs(h.astype(np.float32)) > np.abs(x)
    return np.where(over, np.nextafter(h, np.float16(0)), h).astype(np.float64)


def split2h(x, scale, rnd):
    x = (np.asarray(x, dtype=np.float32).astype(np.float64) * scale).astype(np.float32).astype(np.float64)
    a = rnd(x)
    return [a, rnd(x - a)]


def emul(A, B, pairs=((0, 0), (0, 1), (1, 0), (0, 2), (1, 1), (2, 0)), kc=16, order="small_first"):
    """A [M, N], B [N, C] (already split lists), one fp32 accumulator, chunk = kc."""
    M, N = A[0].shape
    acc = np.zeros((M, B[0].shape[1]), dtype=np.float32)
    pl = list(pairs)
    if order == "small_first":
        pl = pl[::-1]
    for k0 in range(0, N, kc):
        for (i, j) in pl:
            ch = A[i][:, k0:k0 + kc] @ B[j][k0:k0 + kc]  # exact in f64 (8-bit × 8-bit, 16 terms)
            acc = (acc.astype(np.float64) + ch).astype(np.float32)
    return acc.astype(np.float64)


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
    L = np.linalg.cholesky(E11)
    Lit = sl.solve_triangular(L, np.eye(len(E11)), lower=True).T  # L⁻ᵀ [N, N]
    R = float(g.R)
    k0 = R ** 3
    X1d = g.X1.numpy()
    d = tips[:, None, :] - X1d[None, :, :]
    r2 = (d * d).sum(-1)
    r = np.sqrt(r2)
    K = 2 * r2 * r - 3 * R * r2 + R ** 3                                 # [M, N] f64
    V = K @ Lit
    s2 = k0 - (V * V).sum(1)
    s24 = s2.reshape(-1, 4)
    amax = s24.argmax(1)
    d32 = d.astype(np.float32)
    r2f = (d32 * d32).sum(-1, dtype=np.float32)
    rf = np.sqrt(r2f)
    Kf = (np.float32(2) * r2f * rf - np.float32(3 * R) * r2f + np.float32(R ** 3)).astype(np.float64)
    Bs = split3(Lit)
    variants = {
        "K* f64→fp32": (split3(K), 0.0),
        "K* fp32 arith": (split3(Kf), 0.0),
        "K*−R³ f64→fp32": (split3(K - R ** 3), 1.0),
        "K*−R³ fp32 arith": (split3((np.float32(2) * r2f * rf - np.float32(3 * R) * r2f).astype(np.float64)), 1.0),
    }
    colsum = R ** 3 * Lit.sum(0)
    SA = 2.0 ** (10 - np.ceil(np.log2(k0)))
    cm = np.abs(Lit).max(0)
    cm[cm == 0] = 1
    SB = 2.0 ** (14 - np.ceil(np.log2(cm)))[None, :]
    Af16 = (r2f * (np.float32(2 * SA) * rf - np.float32(3 * R * SA))).astype(np.float64)
    results = {name: emul(As, Bs) + off * colsum for name, (As, off) in variants.items()}
    results["fp16 x2 (kernel)"] = (emul(split2h(Af16, 1.0, f16rtz), split2h(Lit, SB, f16), pairs=((0, 0), (0, 1), (1, 0)))
                                   / (SA * SB) + colsum)
    A2, B2 = split2h(Af16, 1.0, f16rtz), split2h(Lit, SB, f16)
    results["fp16 x1 (a0·b0)"] = emul(A2, B2, pairs=((0, 0),)) / (SA * SB) + colsum
    results["fp16 a0·(b0+b1)"] = emul(A2, B2, pairs=((0, 0), (0, 1))) / (SA * SB) + colsum
    results["fp16 (a0+a1)·b0"] = emul(A2, B2, pairs=((0, 0), (1, 0))) / (SA * SB) + colsum
    for name, Ve in results.items():
        s2e = k0 - (Ve * Ve).sum(1)
        err = np.abs(s2e - s2) / k0
        msg = f"{name:18s} |Δstd²|/k0 max {err.max():.2e} p99 {np.percentile(err, 99):.2e}"
        s2e4 = s2e.reshape(-1, 4)
        for mult in (2, 4, 8, 16):
            delta = mult * err.max() * k0
            cand = (s2e4 + delta) >= (s2e4 - delta).max(1, keepdims=True)
            ok = cand[np.arange(len(amax)), amax].all()
            msg += f" | {mult}x: {cand.sum(1).mean():.3f} tips, argmax kept {ok}"
        print(msg, flush=True)


if __name__ == "__main__":
    main()
