// Stream-level launchers of the GPIS std path shared by cdx_gpis_std and the closure
// (defined in cdx_gpis.hip).  ws buffers are caller-owned, sized by the *_ws_bytes helpers.
#pragma once
#include <hip/hip_runtime.h>

#include "cdx.h"

namespace cdx {
size_t gpis_var_ws_bytes(const cdx_gpis& g, int64_t M);
size_t gpis_grad_ws_bytes(const cdx_gpis& g, int64_t M);
// Bytes of the stored whitened vectors V = (L⁻¹K*ᵀ)ᵀ of M queries ([round_up(M, 128), N_pad] f64).
size_t gpis_v_bytes(const cdx_gpis& g, int64_t M);
// Per-group argmax selection fused into the std finalize: rows [t·T, t·T + T) form group t; sel[t]
// = the row of the first maximum of log(100·std) in the group (optimize_pregrasp.py:730's max),
// Xg[t] = X[sel[t]].
struct VarSelect {
  int T;
  int64_t* sel;
  double* Xg;
};
// std[m] = sqrt|k0 − ‖L⁻¹k(x_m)‖²|, var_out[m] = the signed k0 − ‖L⁻¹k‖² (nullable); vout
// (nullable, gpis_v_bytes) receives V; vs (nullable; M a multiple of vs->T) selects per group.
int gpis_var_launch(const cdx_gpis& g, const double* X, int64_t M, double* std_out, double* var_out, void* ws,
                    hipStream_t s, double* vout = nullptr, const VarSelect* vs = nullptr);
// gstd[sel[m]] = ∇std at X[m] (sel null: identity), scaled by var[sel[m]] from gpis_var_launch.
// vin null: W = E11⁻¹k (2N² flops per query); vin = the V of gpis_var_launch: W = L⁻ᵀ v from row
// sel[m] of V (N² flops per query; needs g.Linv).
// vrow (nullable): the V row of query m is vrow[m] instead of sel[m] (the refine pass's list positions).
// fold (nullable, with vin): the finalize is left to the consumer — *fold receives what it needs to
// sum the ∇std pieces of query m itself (grad_fold_gstd), and gstd is not written.
struct GradFold;
int gpis_grad_launch(const cdx_gpis& g, const double* X, int64_t M, const int64_t* sel, const double* var,
                     double* gstd, void* ws, hipStream_t s, const double* vin = nullptr,
                     const int64_t* vrow = nullptr, GradFold* fold = nullptr);

// The ∇std pass's piece partials of a GRADV launch (gpis_std_kernel<GRADV>: each query tile's K-step
// sequence cut into `parts` equal pieces, piece p writing slot p + nt for every stripe nt it touches) and
// the finalize's arithmetic, for a consumer that sums them in its own kernel (the closure's level kernel:
// one launch fewer).  Same slots, same order, same operations as gpis_grad_finalize: bit-identical.
__device__ __host__ inline int grad_fold_ksteps(int nt, int N) {  // gradv_ksteps (256-column stripes, 16-row K-steps)
  const int lo = nt * 256;
  return N > lo ? (N - lo + 15) / 16 : 0;
}

// Cost-balanced pieces of a ∇std (GRADV) query tile (CDX_GRAD_COSTCUT builds; default: equal K-steps).
// The first K-steps of each stripe's range are cheap — the column waves before their diagonal block skip
// their MFMAs (1, 2, 3 blocks, then 4) — so pieces of equal K-steps are not equal in MFMA work; the
// refine pass's measured model (21 + 2·blocks of the busiest SIMD per K-step, RC_FIX / RC_BLK) predicts
// 3.5 % of imbalance here, but cutting by it made the pass slower (0.295 vs 0.286 ms,
// profiles/r03w_cuts_ab.jsonl): the ∇std pass streams V instead of generating K*, its fixed cost per
// K-step is another.  gradv_cut cuts the tile's sequence at equal cost from per-stripe unit costs the
// launcher computes on the host (≤ GC_MAX_NT stripes, indexed statically so that a kernel-argument table
// stays in scalar registers); with none (n = 0) it is the equal-K-step cut.
constexpr int GC_MAX_NT = 16, GC_FIX = 21, GC_BLK = 2;
__device__ __host__ inline int gradv_step_blocks(int s) {  // local step s of a stripe (from its first row)
  int b[4];
  for (int c = 0; c < 4; ++c) {
    const int d = s - 4 * c;
    b[c] = d < 0 ? 0 : (d <= 2 ? d + 1 : 4);
  }
  const int x = b[0] + b[3], y = b[1] + b[2];
  return x > y ? x : y;
}
__device__ __host__ inline int64_t gradv_unit_cost(int nt, int N) {
  const int ks = grad_fold_ksteps(nt, N), nd = ks < 15 ? ks : 15;
  int64_t c = (int64_t)(ks - nd) * (GC_FIX + 8 * GC_BLK);
  for (int s = 0; s < nd; ++s) c += GC_FIX + GC_BLK * gradv_step_blocks(s);
  return c;
}
struct GradCosts {
  int n = 0;                  // stripes with costs (= Nt), 0: equal K-step cuts
  int64_t uc[GC_MAX_NT] = {};
};
// start of piece p of `parts` over the W K-steps of a tile's stripes; uc: the n per-stripe costs (an
// array indexed statically — a kernel argument's member stays in scalar registers)
template <class UC>
__device__ __host__ inline int gradv_cut(int p, int parts, int W, int N, int Nt, const UC& uc, int n) {
  if (p <= 0) return 0;
  if (p >= parts) return W;
  // (short pieces: equal K-steps — a one-step overshoot would cost more than the balance gains)
  if (n != Nt || W < 32 * parts) return (int)((int64_t)W * p / parts);
  int64_t ctot = 0;
#pragma unroll
  for (int nt = 0; nt < GC_MAX_NT; ++nt)
    if (nt < Nt) ctot += uc[nt];
  const int64_t target = ctot * p;  // cost·parts against ctot·p
  int64_t acc = 0;
  int pos = 0;
#pragma unroll
  for (int nt = 0; nt < GC_MAX_NT; ++nt) {
    if (nt >= Nt) break;
    const int ks = grad_fold_ksteps(nt, N);
    if ((acc + uc[nt]) * parts < target) {
      acc += uc[nt];
      pos += ks;
      continue;
    }
    // the stripe's first (diagonal) steps one by one, then its full steps in closed form
    int64_t cum = acc * parts;
    const int nd = ks < 15 ? ks : 15;
    int s = 0;
    while (s < nd && cum < target) cum += (int64_t)(GC_FIX + GC_BLK * gradv_step_blocks(s++)) * parts;
    if (cum < target) {
      const int64_t full = (int64_t)(GC_FIX + 8 * GC_BLK) * parts;
      const int64_t more = (target - cum + full - 1) / full;
      s += (int)(more < ks - s ? more : ks - s);
    }
    return pos + s;
  }
  return W;
}

constexpr int GF_MAX_SLOTS = 32;
struct GradFold {
  const double* partial = nullptr;  // [slots][M_pad][4]
  int64_t M_pad = 0;
  int parts = 0, W = 0, Nt = 0, N = 0;
  GradCosts gc;
  // the slots the pieces wrote, in the order the loop below visits them (host-computed by the launcher; 0: none
  // listed, the consumer walks the cuts itself)
  int n_slots = 0;
  unsigned short slot[GF_MAX_SLOTS] = {};
};
// gstd (3) of query m scaled by the signed variance v: −sign(v)/sqrt|v| · Σ_slots partial[slot][m][1..3]
// (all indices uniform: scalar integer work, the 2·(parts + Nt) loads issued together).
__device__ inline void grad_fold_gstd(const GradFold& f, int64_t m, double v, double* out) {
  double g0 = 0, g1 = 0, g2 = 0;
  if (f.n_slots > 0) {  // the listed slots: the same sums in the same order, without the cut arithmetic
#pragma unroll
    for (int i = 0; i < GF_MAX_SLOTS; ++i) {
      if (i >= f.n_slots) break;
      const double* pp = f.partial + ((int64_t)f.slot[i] * f.M_pad + m) * 4;
      g0 += pp[1]; g1 += pp[2]; g2 += pp[3];
    }
    const double sg = v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0);
    const double fct = -sg / sqrt(fabs(v));
    out[0] = fct * g0; out[1] = fct * g1; out[2] = fct * g2;
    return;
  }
  int q0 = 0;
  for (int p = 0; p < f.parts; ++p) {
    const int q1 = gradv_cut(p + 1, f.parts, f.W, f.N, f.Nt, f.gc.uc, f.gc.n);
    for (int nt = 0, s0 = 0; nt < f.Nt && s0 < q1; ++nt) {
      const int s1 = s0 + grad_fold_ksteps(nt, f.N);
      if (q0 < s1 && s0 < s1) {
        const double* pp = f.partial + ((int64_t)(p + nt) * f.M_pad + m) * 4;
        g0 += pp[1]; g1 += pp[2]; g2 += pp[3];
      }
      s0 = s1;
    }
    q0 = q1;
  }
  const double sg = v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0);
  const double fct = -sg / sqrt(fabs(v));
  out[0] = fct * g0; out[1] = fct * g1; out[2] = fct * g2;
}
// Refine pass behind the split-precision screen: the whitened fp64 pass (V = K*·L⁻ᵀ, Σ V²) for the
// rows rows[0 .. G + *extra) of X (device-side count, at most Mcap), cut into pieces of equal estimated
// cost (one per CU) whatever the count; V rows go to vout at the list positions ([round_up(Mcap, 128),
// N_pad]), Σ V² per (stripe, position) to the returned partial [N_pad/256][*M_pad_out].
// rows null: the identity list (rows 0 .. G + *extra; extra nullable = 0).  gate (nullable): the
// closure's screen statistics — the launch runs only when a check failed (cdx::screen_failed), else every
// workgroup returns at once (the closure's repair pass).  prof: mark the launch for cdx_profile_read.
// after_refine (nullable): recorded on s between the refine kernel and its merge.
// repair (nullable; with gate = its stats, the identity list and G = repair->G·T rows): the closure's
// repair pass — every all-tip row in whole units, then, by the last workgroup, the unscreened selection
// (exact std / var of all rows, sel / vrow / Xg = each group's first maximum of log(100·std)); sets
// SS_REPAIR and counts it.  One gated launch (no merge, no separate selection kernel).
struct RepairSel {
  bool on = false;
  const double* X = nullptr;
  int64_t G = 0;
  int T = 0;
  double *std_ = nullptr, *var = nullptr, *Xg = nullptr;
  int64_t *sel = nullptr, *vrow = nullptr;
  int* stats = nullptr;
  int* done = nullptr;  // (set by the launcher: the workspace's arrival counter)
};
size_t gpis_refine_ws_bytes(const cdx_gpis& g, int64_t Mcap);
// Zeroes the refine workspace's cut-unit arrival counters (once after allocation; every launch
// leaves them zero).
int gpis_refine_reset(const cdx_gpis& g, int64_t Mcap, void* ws, hipStream_t s);
int gpis_refine_launch(const cdx_gpis& g, const double* X, const int* rows, const int* extra, int G, int64_t Mcap,
                       void* ws, double* vout, hipStream_t s, double** partial_out, int64_t* M_pad_out,
                       const int* gate = nullptr, bool prof = true, hipEvent_t after_refine = nullptr,
                       const RepairSel* repair = nullptr);
}  // namespace cdx
