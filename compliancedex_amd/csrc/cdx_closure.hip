// Prob-mode closure on gfx950: FK + query generation, GPIS queries, fused cost+backward.
//
// Launch sequence of cdx_closure (all on the caller's stream, no host sync):
//   1. closure_queries_kernel   one thread per candidate: f32 FK of the pregrasp tips,
//                               palm transform, writes every GPIS query point
//                               (all-tip rows deduplicated over identical coefficient rows,
//                               targets once, pregrasp tips, palm)      — :657-669, :743-750
//   2. gpis_mean (cdx_gpis.hip) mean/∇mean/normal at all queries      — gpis.py:43-87
//   3. gpis std  (cdx_gpis.hip) std at the all-tip queries (whitened, triangular fp64 MFMA,
//      V = L⁻¹k kept; the finalize also selects the variance cost's argmax fingertip),
//      ∇std at those queries only: E11⁻¹k = L⁻ᵀv from the kept V (triangular fp64 MFMA)
//   4. closure_cost_kernel      one thread per candidate: seven cost terms per level,
//                               Kabsch + SVD backward, FK backward; writes loss, margin
//                               and the five parameter gradients        — :713-769, :49-118
#include <hip/hip_runtime.h>

#include "cdx_ab.h"

#include <atomic>
#include <cstdlib>

#include "cdx_collision.h"
#include "cdx_cost.h"
#include "cdx_gpis_launch.h"
#include "cdx_prof.h"
#include "cdx_screen.h"

namespace {

// --------------------------------------------------------------- standalone FK
// One thread per (row, tip): the tip's path is walked with a running pose (no per-thread arrays).
__global__ __launch_bounds__(64) void fk_forward_kernel(cdx_chain c, const float* __restrict__ q, int64_t B,
                                                        float* __restrict__ pos, float* __restrict__ quat) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * c.n_tips) return;
  const int64_t b = t / c.n_tips;
  const int k = (int)(t - b * c.n_tips);
  float p[3], qt[4];
  cdx::fk_tip(c, k, q + b * c.n_dofs, p, qt);
  for (int i = 0; i < 3; ++i) pos[t * 3 + i] = p[i];
  if (quat)
    for (int i = 0; i < 4; ++i) quat[t * 4 + i] = qt[i];
}

// One thread per row: the tips' contributions accumulate into the row of grad_q in tip order.
template <int MAXD>
__global__ __launch_bounds__(64) void fk_backward_kernel(cdx_chain c, const float* __restrict__ q, int64_t B,
                                                         const float* __restrict__ gpos, float* __restrict__ gq) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float* g = gq + b * c.n_dofs;
  for (int i = 0; i < c.n_dofs; ++i) g[i] = 0.f;
  // (the chain read in place from the kernel-argument segment — the first argument, offset 0: indexed per body, the
  // by-value copy went to scratch in the deep-chain instantiation)
  const cdx_chain& kc = *(const cdx_chain*)(__builtin_amdgcn_kernarg_segment_ptr());
  for (int k = 0; k < c.n_tips; ++k)
    cdx::fk_tip_bwd<MAXD>(kc, k, q + b * c.n_dofs, gpos + (b * c.n_tips + k) * 3, cdx::GqAdd{g});
}

// --------------------------------------------------------------- collision loss
__global__ __launch_bounds__(64) void collision_kernel(cdx_collision C, int64_t E, const double* __restrict__ q,
                                                       const double* __restrict__ palm_pos,
                                                       const double* __restrict__ palm_ori, double* __restrict__ cost,
                                                       double* __restrict__ g_q, double* __restrict__ g_pp,
                                                       double* __restrict__ g_po, int accumulate) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int D = C.chain.n_dofs;
  double c, gq[CDX_MAX_DOFS], gpp[3], gpo[3];
  cdx::collision_candidate(C, q + e * D, palm_pos + 3 * e, palm_ori + 3 * e, c, gq, gpp, gpo);
  if (accumulate) {
    cost[e] += c;
    for (int i = 0; i < D; ++i) g_q[e * D + i] += gq[i];
    for (int i = 0; i < 3; ++i) { g_pp[3 * e + i] += gpp[i]; g_po[3 * e + i] += gpo[i]; }
  } else {
    cost[e] = c;
    for (int i = 0; i < D; ++i) g_q[e * D + i] = gq[i];
    for (int i = 0; i < 3; ++i) { g_pp[3 * e + i] = gpp[i]; g_po[3 * e + i] = gpo[i]; }
  }
}

// --------------------------------------------------------------- closure stages
// One thread per (candidate, fingertip): the tip's f32 FK, palm transform (pregrasp_tips, same
// arithmetic), and that fingertip's query points.
__global__ __launch_bounds__(64) void closure_queries_kernel(cdx_problem P, int64_t E, const double* __restrict__ q,
                                                             const double* __restrict__ target,
                                                             const double* __restrict__ palm_pos,
                                                             const double* __restrict__ palm_ori,
                                                             double* __restrict__ X, double* __restrict__ pre_out) {
  const int T = P.chain.n_tips, D = P.chain.n_dofs, Lq = P.n_query_levels;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * T) return;
  const int64_t e = t / T;
  const int f = (int)(t - e * T);
  if (P.loop && t == 0) {  // advance the device loop counters (read by the later kernels)
    P.loop->seed += 1;
    P.loop->step += 1;
  }
  double Rp[9];
  cdx::euler_xyz(palm_ori + 3 * e, Rp, nullptr, nullptr, nullptr);
  float tl[3];
  cdx::fk_tip(P.chain, f, cdx::QRowD{q + e * D}, tl, nullptr);
  double tip[3];
  {
    const double v[3] = {(double)tl[0], (double)tl[1], (double)tl[2]};
    cdx::mat3_vec(Rp, v, tip);
    for (int i = 0; i < 3; ++i) tip[i] = tip[i] + palm_pos[3 * e + i];
  }
  const double* tg = target + (e * T + f) * 3;
  for (int u = 0; u < Lq; ++u) {
    int k = 0;
    while (k < P.n_levels - 1 && P.level_query[k] != u) ++k;
    const double c = (double)P.coeff[k][f];
    const int64_t qi = cdx::q_alltip(u, e, f, E, T);
    for (int i = 0; i < 3; ++i) X[3 * qi + i] = tg[i] + c * (tip[i] - tg[i]);
  }
  const int64_t qt = cdx::q_target(Lq, e, f, E, T), qp = cdx::q_pre(Lq, e, f, E, T);
  for (int i = 0; i < 3; ++i) {
    X[3 * qt + i] = tg[i];
    X[3 * qp + i] = tip[i];
    if (pre_out) pre_out[(e * T + f) * 3 + i] = tip[i];
  }
  if (P.optimize_palm && f == 0) {
    const int64_t qm = cdx::q_palm(Lq, e, E, T);
    for (int i = 0; i < 3; ++i) X[3 * qm + i] = palm_pos[3 * e + i];
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct GpisView {
  const double *mean, *gmean, *normal, *std_, *gstd;
  int64_t E;
  int T, Lq;
  __device__ cdx::GpisPoint operator()(int kind, int u, int f) const;
  int64_t e;
  // ∇std folded into the level kernel (screened closure): the kernel sums its group's ∇std from the pass's
  // piece partials once (cdx::grad_fold_gstd with sel / var) into gsv, the value of all-tip row gq
  cdx::GradFold fold;
  const double* var = nullptr;
  const int64_t* sel = nullptr;
  int64_t gq = -1;
  double gsv[3] = {0, 0, 0};
};

__device__ cdx::GpisPoint GpisView::operator()(int kind, int u, int f) const {
  cdx::GpisPoint p;
  int64_t qi;
  if (kind == 0) qi = cdx::q_alltip(u, e, f, E, T);
  else if (kind == 1) qi = cdx::q_target(Lq, e, f, E, T);
  else if (kind == 2) qi = cdx::q_pre(Lq, e, f, E, T);
  else qi = cdx::q_palm(Lq, e, E, T);
  p.mean = mean[qi];
  for (int i = 0; i < 3; ++i) p.gmean[i] = gmean[3 * qi + i];
  if (kind == 0) {
    p.std = std_[qi];
    for (int i = 0; i < 3; ++i) p.normal[i] = normal[3 * qi + i];
    // (only the group's selected row — the variance cost's argmax — has a ∇std; level_fwd_bwd reads no other)
    if (fold.partial)
      for (int i = 0; i < 3; ++i) p.gstd[i] = qi == gq ? gsv[i] : 0.0;
    else
      for (int i = 0; i < 3; ++i) p.gstd[i] = gstd[3 * qi + i];
  } else {
    p.std = 0;
    for (int i = 0; i < 3; ++i) { p.gstd[i] = 0; p.normal[i] = 0; }
  }
  return p;
}

// Per-(level, candidate) thread: compute_loss of one pregrasp level, forward + backward.
// Record per (k, e): [l, margin[T], g_tip[T][3], g_target[T][3], g_comp[T]]  (1 + 8T doubles).
CDX_HD int level_record_width(int T) { return 1 + 8 * T; }

__device__ __forceinline__ void device_noise(uint64_t seed, int64_t row, double* nz) {
  for (int i = 0; i < 9; ++i) {
    const uint64_t r = splitmix64(seed ^ splitmix64((uint64_t)(row * 9 + i)));
    nz[i] = (double)(r >> 11) * 0x1.0p-53;
  }
}

// --------------------------------------------------------------- force_eq_reward
CDX_HD cdx::ForceEqParams force_eq_params(const cdx_force_eq& p) {
  cdx::ForceEqParams fp;
  fp.cos_mu = (double)p.cos_mu;
  fp.gravity = p.gravity;
  for (int i = 0; i < 3; ++i) fp.com[i] = (double)p.com[i];
  fp.dummy_target_z = (double)p.dummy_target_z;
  fp.dummy_comp = (double)p.dummy_comp;
  return fp;
}

template <int NT>
__device__ __forceinline__ void force_eq_row(const cdx_force_eq& p, int64_t b, const double* tip,
                                             const double* target, const double* comp, const double* normal,
                                             const double* noise, uint64_t seed, cdx::ForceEq<NT>& fe) {
  constexpr int NTA = cdx::ForceEq<NT>::NTA;
  const int T = NT > 0 ? NT : p.n_tips;
  double tp[NTA][3], nr[NTA][3], nz[9];
  for (int f = 0; f < T; ++f)
    for (int i = 0; i < 3; ++i) { tp[f][i] = tip[(b * T + f) * 3 + i]; nr[f][i] = normal[(b * T + f) * 3 + i]; }
  if (noise) {
    for (int i = 0; i < 9; ++i) nz[i] = noise[b * 9 + i];
  } else {
    device_noise(seed, b, nz);
  }
  fe.forward(force_eq_params(p), T, tp, target + b * T * 3, comp + b * T, nr, nz);
}

template <int NT>
__global__ __launch_bounds__(64) void force_eq_forward_kernel(cdx_force_eq p, int64_t B, const double* __restrict__ tip,
                                                              const double* __restrict__ target,
                                                              const double* __restrict__ comp,
                                                              const double* __restrict__ normal,
                                                              const double* __restrict__ noise, uint64_t seed,
                                                              double* __restrict__ reward, double* __restrict__ margin,
                                                              double* __restrict__ force_norm, int32_t* __restrict__ flip) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  cdx::ForceEq<NT> fe;
  force_eq_row<NT>(p, b, tip, target, comp, normal, noise, seed, fe);
  const int T = NT > 0 ? NT : p.n_tips;
  reward[b] = fe.reward;
  for (int f = 0; f < T; ++f) { margin[b * T + f] = fe.margin[f]; force_norm[b * T + f] = fe.fn[f]; }
  if (flip) flip[b] = fe.flip;
}

template <int NT>
__global__ __launch_bounds__(64) void force_eq_backward_kernel(
    cdx_force_eq p, int64_t B, const double* __restrict__ tip, const double* __restrict__ target,
    const double* __restrict__ comp, const double* __restrict__ normal, const double* __restrict__ noise, uint64_t seed,
    const double* __restrict__ g_reward, const double* __restrict__ g_force_norm, double* __restrict__ g_tip,
    double* __restrict__ g_target, double* __restrict__ g_comp) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  cdx::ForceEq<NT> fe;
  force_eq_row<NT>(p, b, tip, target, comp, normal, noise, seed, fe);
  constexpr int NTA = cdx::ForceEq<NT>::NTA;
  const int T = NT > 0 ? NT : p.n_tips;
  double gfn[NTA], gt[NTA][3], gg[NTA][3], gc[NTA];
  for (int f = 0; f < T; ++f) {
    gfn[f] = g_force_norm ? g_force_norm[b * T + f] : 0.0;
    gt[f][0] = gt[f][1] = gt[f][2] = 0.0;
    gg[f][0] = gg[f][1] = gg[f][2] = 0.0;
    gc[f] = 0.0;
  }
  fe.backward(g_reward ? g_reward[b] : 0.0, gfn, comp + b * T, gt, gg, gc);
  for (int f = 0; f < T; ++f) {
    for (int i = 0; i < 3; ++i) { g_tip[(b * T + f) * 3 + i] = gt[f][i]; g_target[(b * T + f) * 3 + i] = gg[f][i]; }
    g_comp[b * T + f] = gc[f];
  }
}

template <int NT, int G, bool PRE = false, bool VL = false>
__global__ __launch_bounds__(64) void closure_level_kernel(cdx_problem P, int64_t E, const double* __restrict__ q,
                                                           const double* __restrict__ comp,
                                                           const double* __restrict__ target,
                                                           const double* __restrict__ X,
                                                           const double* __restrict__ noise, uint64_t seed,
                                                           GpisView gv, double* __restrict__ lvl,
                                                           int32_t* __restrict__ flip,
                                                           const double* __restrict__ krot) {
#if defined(CDX_LEVEL_PRIO)
  // latency-bound dependent chains: issue first whenever ready, so that the GPIS mean's part B on
  // the side stream (CDX_MEAN_SPLIT) fills the issue slots the chains leave without stretching them
  __builtin_amdgcn_s_setprio(CDX_LEVEL_PRIO);
#endif
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int K = P.n_levels;
  if (t >= K * E) return;
  const int k = (int)(t / E);
  const int64_t e = t - (int64_t)k * E;
  const int T = NT > 0 ? NT : P.chain.n_tips, D = P.chain.n_dofs, Lq = P.n_query_levels;
  double tip[CDX_MAX_TIPS][3];
  for (int f = 0; f < T; ++f)
    for (int i = 0; i < 3; ++i) tip[f][i] = X[3 * cdx::q_pre(Lq, e, f, E, T) + i];
  double nz[9];
  cdx::CandidateIn in;
  in.q = q + e * D;
  in.comp = comp + e * T;
  in.target = target + e * T * 3;
  in.palm_pos = in.palm_ori = nullptr;
  // the draw is copied into registers either way: a pointer that may address either global memory
  // or this array would keep nz in scratch
  if (noise) {
    for (int i = 0; i < 9; ++i) nz[i] = noise[t * 9 + i];
  } else {
    device_noise(P.loop ? seed ^ splitmix64(P.loop->seed) : seed, t, nz);
  }
  in.noise = nz;
  in.noise_stride = 0;
  in.rot = krot ? krot + t * cdx::ForceEq<NT, G>::KABSCH_RECORD : nullptr;
  double dq[CDX_MAX_DOFS];
  const double qnorm = cdx::ref_dist(P, in.q, dq);
  GpisView g = gv;
  g.e = e;
  if (!VL && gv.fold.partial) {  // this level's group: its selected row and ∇std (the finalize, folded; read
    // from the kernel argument itself: its cost table stays in scalar registers)
    const int64_t m = (int64_t)P.level_query[k] * E + e;
    g.gq = gv.sel[m];
    cdx::grad_fold_gstd(gv.fold, m, gv.var[g.gq], g.gsv);
  }
  cdx::LevelOut lo;
  cdx::level_fwd_bwd<NT, GpisView, G, PRE, !VL>(P, k, in, tip, qnorm, g, lo);
  double* r = lvl + t * level_record_width(T);
  r[0] = lo.l;
  for (int f = 0; f < T; ++f) {
    r[1 + f] = lo.margin[f];
    r[1 + 7 * T + f] = lo.g_comp[f];
    for (int i = 0; i < 3; ++i) {
      r[1 + T + 3 * f + i] = lo.g_tip[f][i];
      r[1 + 4 * T + 3 * f + i] = lo.g_target[f][i];
    }
  }
  if (flip) flip[t] = lo.flip;
}

// Per-(level, candidate) thread: the Kabsch stage of force_eq_reward (:49-69) — the weighted
// cross-covariance of the level's all-tip points and the targets, its 3×3 SVD and the rotation — as a
// record the level kernel loads instead of running the SVD itself (ForceEq::save_rotation).  Its inputs
// are the query points, compliances, targets and the Kabsch noise only (not the GPIS results), so the
// screened closure runs it on the side stream after the screen kernel, beside the latency-bound
// selection and compaction, and takes the SVD (≈ 21 of the level kernel's 45 µs at E = 4096,
// CDX_DIAG_NOSVD build) off the critical path.  Same
// arithmetic as the inline path (both are ForceEq::rotation on the same values): bit-identical records.
template <int NT, int G>
__global__ __launch_bounds__(64) void closure_kabsch_kernel(cdx_problem P, int64_t E, const double* __restrict__ comp,
                                                            const double* __restrict__ target,
                                                            const double* __restrict__ X,
                                                            const double* __restrict__ noise, uint64_t seed,
                                                            double* __restrict__ krot) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int K = P.n_levels;
  if (t >= K * E) return;
  const int k = (int)(t / E);
  const int64_t e = t - (int64_t)k * E;
  const int T = NT > 0 ? NT : P.chain.n_tips, Lq = P.n_query_levels;
  constexpr int NTA = cdx::ForceEq<NT, G>::NTA;
  double a[NTA][3];
  const double* tg = target + e * T * 3;
  for (int f = 0; f < T; ++f) {
    const double c = (double)P.coeff[k][f];  // the all-tip point exactly as level_fwd_bwd forms it
    for (int i = 0; i < 3; ++i) a[f][i] = tg[3 * f + i] + c * (X[3 * cdx::q_pre(Lq, e, f, E, T) + i] - tg[3 * f + i]);
  }
  double nz[9];
  if (noise) {
    for (int i = 0; i < 9; ++i) nz[i] = noise[t * 9 + i];
  } else {
    device_noise(P.loop ? seed ^ splitmix64(P.loop->seed) : seed, t, nz);
  }
  cdx::ForceEq<NT, G> fe;
  fe.setup(cdx::force_eq_params(P), T, a, tg, comp + e * T, nullptr);
  fe.rotation(nz);
  fe.save_rotation(krot + t * cdx::ForceEq<NT, G>::KABSCH_RECORD);
}

// Per-candidate group of GS lanes, lane f = fingertip f: sums the levels, adds the pregrasp
// and palm GPIS terms (:757-763), the palm/euler backward and the fingertip's FK VJP, then
// reduces the shared gradients: palm terms with xor-shuffles, the per-DOF FK contributions
// through LDS ([dof][thread], summed in the same pairwise order over the group's lanes).
// VL (var_late): the level records hold no variance cost; lane f adds it here for the levels whose group
// maximum (sel, the first maximum of log(100·std) as level_fwd_bwd takes it) is fingertip f — loss
// w_k·(l_k + uncertainty·log(100·std)) and, through the all-tip interpolation a = target + c·(tip −
// target), c·g and g − c·g of g = w_k·uncertainty/std·∇std into the tip and target gradients; ∇std
// summed from the pass's pieces here when folded (once per distinct level, by that fingertip's lane).
#if !defined(CDX_COMBINE_BLOCK)
#define CDX_COMBINE_BLOCK 64
#endif
constexpr int COMBINE_BLOCK = CDX_COMBINE_BLOCK;  // 64: E = 4096 spreads over 256 workgroups, one per CU
template <int GS, int MAXD, bool VL = false>
__global__ __launch_bounds__(COMBINE_BLOCK) void closure_combine_kernel(
    cdx_problem P, int64_t E, const double* __restrict__ q, const double* __restrict__ palm_pos,
    const double* __restrict__ palm_ori, GpisView gv, const double* __restrict__ lvl, double* __restrict__ total_loss,
    double* __restrict__ total_margin, double* __restrict__ g_q, double* __restrict__ g_comp,
    double* __restrict__ g_target, double* __restrict__ g_palm_pos, double* __restrict__ g_palm_ori) {
  __shared__ float gcon[CDX_MAX_DOFS][COMBINE_BLOCK];
  const int tid = threadIdx.x;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + tid;
  const int64_t e = gid / GS;
  const int f = (int)(gid % GS);
  const int T = P.chain.n_tips, D = P.chain.n_dofs, K = P.n_levels;
  const bool valid = e < E;
  const bool live = valid && f < T;
  const int LW = level_record_width(T);
  const int64_t ec = valid ? e : 0;
  GpisView g = gv;
  g.e = ec;

  double gt[3] = {0, 0, 0}, gtar[3] = {0, 0, 0}, gcomp = 0, marg = 0;
  double total = 0.0;  // Σ_k w_k·l_k (lane 0's)
  if (live) {
    int ulast = -1;
    int64_t qsel = -1;
    double gs3[3] = {0, 0, 0}, ssel = 0, lsel = 0;
    for (int k = 0; k < K; ++k) {
      const double* r = lvl + ((int64_t)k * E + e) * LW;
      marg += P.weight[k] * r[1 + f];
      gcomp += r[1 + 7 * T + f];
      for (int i = 0; i < 3; ++i) { gt[i] += r[1 + T + 3 * f + i]; gtar[i] += r[1 + 4 * T + 3 * f + i]; }
      double l = r[0];
      if constexpr (VL) {
        const int u = P.level_query[k];
        if (u != ulast) {  // this distinct level's group maximum and (on its lane) its ∇std
          ulast = u;
          const int64_t m = (int64_t)u * E + e;
          qsel = gv.sel[m];
          ssel = gv.std_[qsel];
          lsel = log(100 * ssel);  // the level loss's max_f log(100·std_f)
          if (qsel == cdx::q_alltip(u, e, f, E, T)) {
#if defined(CDX_COMBINE_DIAG_NOFOLD)  // (timing-only diagnostic build: outputs wrong)
            if (false)
#else
            if (gv.fold.partial)
#endif
              cdx::grad_fold_gstd(gv.fold, m, gv.var[qsel], gs3);
            else
              for (int i = 0; i < 3; ++i) gs3[i] = gv.gstd[3 * qsel + i];
          }
        }
        if (qsel == cdx::q_alltip(u, e, f, E, T)) {
          const double gs = P.weight[k] * P.uncertainty / ssel, c = (double)P.coeff[k][f];
          for (int i = 0; i < 3; ++i) {
            const double ga = gs * gs3[i];
            gt[i] += c * ga;
            gtar[i] += ga - c * ga;
          }
        }
        l = l + P.uncertainty * lsel;
      }
      total += P.weight[k] * l;
    }
    const cdx::GpisPoint gpp = g(2, 0, f);
    for (int i = 0; i < 3; ++i) gt[i] += -5.0 * gpp.gmean[i];
  }
  // palm transform backward: tip = Rp·tl + palm_pos
  double Rp[9], dRa[9], dRb[9], dRc[9];
  cdx::euler_xyz(palm_ori + 3 * ec, Rp, dRa, dRb, dRc);
  double gl[3];
  cdx::mat3t_vec(Rp, gt, gl);
  const float gtl[3] = {(float)gl[0], (float)gl[1], (float)gl[2]};
  for (int i = 0; i < D; ++i) gcon[i][tid] = 0.f;
  float tl[3] = {0.f, 0.f, 0.f};
  if (live) {
    // the chain read in place from the kernel-argument segment (P is the first argument, at offset 0)
    const cdx_chain& kc = (*(const cdx_problem*)(__builtin_amdgcn_kernarg_segment_ptr())).chain;
#if defined(CDX_COMBINE_FK_BWD1)  // (A/B: the stored-rotations backward walk)
    cdx::fk_tip_bwd<MAXD>(kc, f, cdx::QRowD{q + ec * D}, gtl, [&](int d, float v) { gcon[d][tid] += v; }, tl);
#elif defined(CDX_COMBINE_FK_BWD3R)  // (A/B: round 5 — one unrolled walk in registers for the hands, two walks for deep
                                     // chains)
    if constexpr (MAXD <= 8)
      cdx::fk_tip_bwd3<MAXD>(kc, f, cdx::QRowD{q + ec * D}, gtl, [&](int d, float v) { gcon[d][tid] += v; }, tl);
    else
      cdx::fk_tip_bwd2<MAXD>(kc, f, cdx::QRowD{q + ec * D}, gtl, [&](int d, float v) { gcon[d][tid] += v; }, tl);
#elif !defined(CDX_COMBINE_DIAG_NOFK)  // (timing-only diagnostic build without the FK backward: outputs wrong)
    // one rolled walk, the joints' axes and origins in LDS, then the per-joint products (fk_tip_bwd3's arithmetic;
    // deep chains no longer walk twice)
    __shared__ float s_cst[6 * MAXD * COMBINE_BLOCK];
    float R[9], t[3];
    cdx::fk_tip_walk3s(kc, f, cdx::QRowD{q + ec * D}, R, t,
                       [&](int l, int i, float v) { s_cst[(6 * l + i) * COMBINE_BLOCK + tid] = v; });
    cdx::tip_from_pose(kc, f, R, t, tl, nullptr);
    cdx::fk_tip_bwd3_grad(kc, f, R, t, gtl, [&](int d, float v) { gcon[d][tid] += v; },
                          [&](int l, int i) { return s_cst[(6 * l + i) * COMBINE_BLOCK + tid]; });
#endif
  }
  double red[12];  // g_palm_pos (3) + g_Rp (9)
  for (int i = 0; i < 3; ++i) red[i] = gt[i];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) red[3 + 3 * r + c] = gt[r] * (double)tl[c];
#pragma unroll
  for (int m = 1; m < GS; m <<= 1)
    for (int i = 0; i < 12; ++i) red[i] += __shfl_xor(red[i], m);
  __syncthreads();
  if (!valid) return;
  // g_q = ref-distance term + Σ_lanes FK contributions; lane f takes DOFs f, f + GS, ...
  double qn2 = 0.0;
  for (int i = 0; i < D; ++i) {
    const double dq = q[e * D + i] - (double)P.ref_q[i];
    qn2 += dq * dq;
  }
  const double qnorm = sqrt(qn2);
  const int base = tid - f;
  for (int i = f; i < D; i += GS) {
    double s[GS];
#pragma unroll
    for (int j = 0; j < GS; ++j) s[j] = (double)gcon[i][base + j];
#pragma unroll
    for (int w = 1; w < GS; w <<= 1)
#pragma unroll
      for (int j = 0; j < GS; j += 2 * w) s[j] += s[j + w];
    const double dq = q[e * D + i] - (double)P.ref_q[i];
    double v = 0.0;
    if (qnorm > 0)
      for (int k = 0; k < K; ++k) v += P.weight[k] * 10.0 * dq / qnorm;
    g_q[e * D + i] = v + s[0];
  }
  if (live) {
    total_margin[e * T + f] = marg;
    g_comp[e * T + f] = gcomp;
    for (int i = 0; i < 3; ++i) g_target[(e * T + f) * 3 + i] = gtar[i];
  }
  if (f != 0) return;
  double pre_sum = 0.0;
  for (int ff = 0; ff < T; ++ff) pre_sum += g(2, 0, ff).mean;
  total = total - pre_sum * 5.0;
  double gpp[3] = {red[0], red[1], red[2]};
  if (P.optimize_palm) {
    const cdx::GpisPoint gpm = g(3, 0, 0);
    total = total + 1.0 / gpm.mean;
    const double gm = -1.0 / (gpm.mean * gpm.mean);
    for (int i = 0; i < 3; ++i) gpp[i] = gm * gpm.gmean[i] + gpp[i];
  }
  total_loss[e] = total;
  double go[3] = {0, 0, 0};
  for (int i = 0; i < 9; ++i) {
    go[0] += red[3 + i] * dRa[i];
    go[1] += red[3 + i] * dRb[i];
    go[2] += red[3 + i] * dRc[i];
  }
  for (int i = 0; i < 3; ++i) { g_palm_pos[3 * e + i] = gpp[i]; g_palm_ori[3 * e + i] = go[i]; }
}

bool chain_ok(const cdx_chain* c) {
  if (!(c && c->n_bodies > 0 && c->n_bodies <= CDX_MAX_BODIES && c->n_dofs >= 0 && c->n_dofs <= CDX_MAX_DOFS &&
        c->n_tips > 0 && c->n_tips <= CDX_MAX_TIPS))
    return false;
  // parents precede children (the FK walks a tip's path in ascending body order), DOFs in range
  for (int i = 1; i < c->n_bodies; ++i)
    if (c->bodies[i].parent < 0 || c->bodies[i].parent >= i || c->bodies[i].dof >= c->n_dofs) return false;
  for (int k = 0; k < c->n_tips; ++k)
    if (c->tip_body[k] < 0 || c->tip_body[k] >= c->n_bodies) return false;
  return true;
}

// fk_tip_bwd register bound for a chain: 8 levels (the hands) or CDX_MAX_DEPTH (arm + hand).
bool shallow_chain(const cdx_chain& c) { return cdx::chain_max_depth(c) <= 8; }

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

struct ClosureWs {
  double *X, *mean, *gmean, *normal, *std_, *var, *gstd, *Xg, *lvl, *V;
  double* krot;  // Kabsch records [n_levels·E][KABSCH_RECORD] (screened closure: computed on the side stream)
  int64_t* sel;
  void *var_ws, *grad_ws;
  // split-precision screening (screen_on): estimates, list positions, the kept-row list, per-group
  // keep / audit masks, statistics (cdx::ScreenStat), ∇std V rows, screen / refine scratch
  double* sv2;
  int *vpos, *rows, *stats;
  unsigned* zkey;  // discarded rows' normalised gap z (float bits) for the audit
  unsigned short* keep;
  int64_t* vrow;
  void *screen_ws, *refine_ws;
  size_t bytes;
};

// Where the screened closure forks the GPIS mean onto its side stream (CDX_FORK_MEAN overrides):
//   2 (default): after the screen — the mean fills the CUs the selection / compaction kernels leave
//     idle and shares the machine with the exact pass: 1.156–1.163 vs 1.188–1.200 ms per closure at
//     config 2 unforked (profiles/r02o_fork_point_ab.txt);
//   1: beside the screen — the screen stretched 0.334 → 0.425 ms (bf16 version), net loss
//     (profiles/r02g_fork_mean_ab.txt);  3: after the exact pass, beside the ∇std pass: 1.175 ms;
//   4: after the screen kernel, before its selection / compaction (≈ 30 µs of a nearly idle chip);
//   0: no fork.  Values above 4 are taken as 0.
int fork_point() {
  static const int at = [] {
    const char* e = cdx::ab_env("CDX_FORK_MEAN");
    const int v = e ? std::max(0, atoi(e)) : 2;
    return v > 4 ? 0 : v;
  }();
  return at;
}
bool fork_mean() {
  static const bool on = fork_point() > 0;
  return on;
}

// The closure screens the all-tip rows with the bf16 estimate when the GPIS state carries a
// calibrated screen (cdx_gpis_screen_prepare + screen_delta), CDX_NO_SCREEN is unset and there are
// enough rows to fill the chip: below SCREEN_MIN_ROWS the screen runs a handful of workgroups and
// its fixed cost (five launches) exceeds the fp64 pass it saves (config 1: E = 64, N = 361 runs
// 0.16 ms unscreened on split-K, 1.6 ms screened).
constexpr int64_t SCREEN_MIN_ROWS = 4096;

bool screen_on(const cdx_problem* p, int64_t E) {
#if defined(CDX_GRAD_EXPLICIT)
  return false;  // the screened path keeps V for the ∇std pass, which this build does not allocate
#endif
  static const bool off = cdx::ab_env("CDX_NO_SCREEN") != nullptr;
  const int64_t Ms = (int64_t)p->n_query_levels * E * p->chain.n_tips;
  return !off && p->gpis.screen && p->gpis.screen_delta > 0 && p->chain.n_tips <= CDX_MAX_TIPS &&
         Ms >= SCREEN_MIN_ROWS;
}

// The variance cost takes max_f log(100·std_f) (:730), so ∇std is only ever needed at one
// fingertip per (distinct level, candidate): the std finalize picks it exactly as level_fwd_bwd
// does (first maximum of log(100·s), cdx::VarSelect) and gathers its query for the ∇std GEMM.

ClosureWs closure_ws_layout(const cdx_problem* p, int64_t E, char* base) {
  ClosureWs w;
  const int64_t Mq = cdx::n_queries(*p, E);
  const int64_t Ms = (int64_t)p->n_query_levels * E * p->chain.n_tips;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* r = base ? base + off : nullptr; off += align256(bytes); return r; };
  w.X = (double*)take(Mq * 3 * sizeof(double));
  w.mean = (double*)take(Mq * sizeof(double));
  w.gmean = (double*)take(Mq * 3 * sizeof(double));
  w.normal = (double*)take(Mq * 3 * sizeof(double));
  const int64_t Mg = (int64_t)p->n_query_levels * E;
  w.std_ = (double*)take(Ms * sizeof(double));
  w.var = (double*)take(Ms * sizeof(double));
  w.gstd = (double*)take(Ms * 3 * sizeof(double));
  w.sel = (int64_t*)take(Mg * sizeof(int64_t));
  w.Xg = (double*)take(Mg * 3 * sizeof(double));
  const bool scr = screen_on(p, E);
  w.var_ws = scr ? nullptr : take(cdx::gpis_var_ws_bytes(p->gpis, Ms));
  w.grad_ws = take(cdx::gpis_grad_ws_bytes(p->gpis, Mg));
  w.sv2 = scr ? (double*)take(Ms * sizeof(double)) : nullptr;
  w.vpos = scr ? (int*)take(Ms * sizeof(int)) : nullptr;
  w.rows = scr ? (int*)take(Ms * sizeof(int)) : nullptr;
  w.stats = scr ? (int*)take(cdx::SS_WORDS * sizeof(int)) : nullptr;
  w.zkey = scr ? (unsigned*)take((Ms + cdx::screen_compact_words(Mg)) * sizeof(unsigned)) : nullptr;
  w.keep = scr ? (unsigned short*)take(Mg * sizeof(unsigned short)) : nullptr;
  w.vrow = scr ? (int64_t*)take(Mg * sizeof(int64_t)) : nullptr;
  w.screen_ws = scr ? take(cdx::screen_ws_bytes(p->gpis, Ms)) : nullptr;
  w.refine_ws = scr ? take(cdx::gpis_refine_ws_bytes(p->gpis, Ms)) : nullptr;
  w.lvl = (double*)take((size_t)p->n_levels * E * level_record_width(p->chain.n_tips) * sizeof(double));
  w.krot = scr ? (double*)take((size_t)p->n_levels * E * cdx::ForceEq<0>::KABSCH_RECORD * sizeof(double)) : nullptr;
#if !defined(CDX_GRAD_EXPLICIT)
  w.V = (double*)take(cdx::gpis_v_bytes(p->gpis, Ms));
#else
  w.V = nullptr;
#endif
  w.bytes = off;
  return w;
}

// Side stream of the screened closure (one per device, created on first use): the GPIS mean
// (fp64 VALU-bound, 4-wave workgroups, 96 VGPRs, 8 KB LDS) runs concurrently with the selection and
// exact-pass kernels (fork_point); the level kernel waits for it.  Fork and join are event waits
// (hipGraph-capturable).  Not for concurrent cdx_closure calls from several host threads on one
// device.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;  // main → side before mean A, side → main after it
  hipEvent_t gate = nullptr, joinB = nullptr; // main → side after the ∇std pass, side → main after mean B
  hipEvent_t late = nullptr;                   // main → side after the refine kernel (mean_sched() 4)
  // the split mean schedule (mean_sched() 2): a second side stream for the mean chunks
  hipStream_t s2 = nullptr;
  hipEvent_t g1 = nullptr, g2 = nullptr, e2a = nullptr, jb = nullptr;
};

// Mean schedule of the screened closure (CDX_MEAN_SCHED): 1 (default) the whole mean on the side stream
// after the Kabsch records; 2 the mean in two chunks on a second side stream, each in a window where the
// main stream runs latency- or bandwidth-bound kernels: rows [0, M1) (CDX_MEAN_CHUNK1 of them, default 0.3)
// beside the selection / compaction — the refine pass waits for them —, the rest beside the merge and the
// exact selection after the refine pass; the level kernel follows the all-tip and target rows; 4 the
// whole mean after the refine kernel (the side stream waits an event recorded between it and the merge),
// beside the bandwidth-bound merge and the latency-bound exact selection, instead of whichever of the
// refine pass and the mean the command processor happens to dispatch first after the records.
int mean_sched() {
  static const int m = [] {
    const char* e = cdx::ab_env("CDX_MEAN_SCHED");
    return e ? atoi(e) : 1;
  }();
  return m;
}
// Order on the side stream (CDX_MEAN_FIRST): 0 (round 5 default) the Kabsch records, then mean A; 1 mean A
// first (round 4's default, with the one-workgroup compaction: the mean then started in the window of the
// latency-bound selection and compaction, 1.013 vs 1.036 ms, profiles/r04q_ab_mean_first_side_prio.jsonl).
// With the compaction spread over the chip (screen_count / screen_place kernels, round 5) the mean's
// workgroups arriving first stretch those two kernels instead: records first measured 0.984–0.989 vs
// 0.996–0.998 ms per closure over 3 interleaved rounds (profiles/r05n_ab_side_order.jsonl).
bool mean_first() {
  static const bool on = [] {
    const char* e = cdx::ab_env("CDX_MEAN_FIRST");
    return e && atoi(e) != 0;
  }();
  return on;
}
// CDX_JOIN_EARLY=1: the caller's stream waits for the side stream (records, mean, level kernel) before the ∇std pass
// instead of before the combine kernel — the level kernel ends ≈ 3 µs before the ∇std pass would start, and the
// wait in front of the combine costs ≈ 7 µs of gap (A/B).
bool join_early() {
  static const bool on = [] {
    const char* e = cdx::ab_env("CDX_JOIN_EARLY");
    return e && atoi(e) != 0;
  }();
  return on;
}
double mean_chunk1() {
  static const double f = [] {
    const char* e = cdx::ab_env("CDX_MEAN_CHUNK1");
    const double v = e ? atof(e) : 0.3;
    return v < 0 ? 0.0 : (v > 1 ? 1.0 : v);
  }();
  return f;
}

// CDX_MEAN_SPLIT=1 splits the forked mean: part A — the all-tip and target rows, which the level
// kernel reads — at the fork point; part B — the pregrasp and palm rows, read only by the combine
// kernel — gated behind the ∇std pass, beside the latency-bound level kernel (3E lanes, ≈ 1/5 of the
// SIMDs).  Off by default: 1.135–1.154 vs 1.095–1.110 ms per closure (profiles/r03e_mean_split_ab.jsonl)
// — mean B's waves share SIMDs with the level kernel's long dependent chains and stretch them.
bool mean_split() {
  static const bool on = [] {
    const char* e = cdx::ab_env("CDX_MEAN_SPLIT");
    return e && atoi(e) != 0;
  }();
  return on;
}

// Kabsch records computed ahead of the level kernel (closure_kabsch_kernel), CDX_KABSCH_AHEAD: 1
// (default) on the side stream ahead of the mean, one fork after the screen kernel; 0 the level kernel
// runs the SVD itself.  (A stream of their own, with their own fork / join events, measured 1.24–1.26
// vs 1.05 ms per closure — the refine pass slowed 0.34 → 0.58 ms; profiles/r03t_kabsch_ab.jsonl.)
int kabsch_mode() {
  static const int m = [] {
    const char* e = getenv("CDX_KABSCH_AHEAD");
    return e && atoi(e) == 0 ? 0 : 1;
  }();
  return m;
}

// CDX_GRAD_FOLD=0 keeps the ∇std finalize kernel (A/B); default: the screened closure's level kernel
// sums the ∇std pieces of its group itself (GpisView::fold) — one launch fewer.
bool grad_fold() {
  static const bool on = [] {
    const char* e = cdx::ab_env("CDX_GRAD_FOLD");
    return !e || atoi(e) != 0;
  }();
  return on;
}

// Fork/join events: no timing, and (CDX_SIDE_EVENT_FENCE=0 / unset) no system-scope fence — they order
// two streams of one device, whose kernels see each other's writes at kernel boundaries anyway.
unsigned side_event_flags() {
  static const unsigned f = [] {
    const char* e = cdx::ab_env("CDX_SIDE_EVENT_FENCE");
    return (e && atoi(e) != 0) ? (unsigned)hipEventDisableTiming
                               : (unsigned)(hipEventDisableTiming | hipEventDisableSystemFence);
  }();
  return f;
}

bool side_stream(SideStream& out) {
  static SideStream per_dev[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  SideStream& ss = per_dev[dev];
  if (!ss.s) {
    hipStream_t st;
    // CDX_SIDE_PRIO: < 0 creates the side stream at the device's lowest priority, > 0 at its highest (the
    // CP prefers a higher-priority queue's dispatches; round 3's default, −3…−4 µs then with the records
    // first, profiles/r03zi_side_prio_ab.jsonl, r03zj_side_prio_default_ab.jsonl), 0 normal (round 4
    // default, with the mean first: the highest priority lets the mean's workgroups starve the main
    // stream's compaction; 1.013 vs 1.016 (lowest) vs 1.036 ms (highest, records first),
    // r04q_ab_mean_first_side_prio.jsonl).
    const char* pe = cdx::ab_env("CDX_SIDE_PRIO");
    const int want = pe ? atoi(pe) : 0;
    int least = 0, greatest = 0;
    hipError_t ce;
    if (want != 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      ce = hipStreamCreateWithPriority(&st, hipStreamNonBlocking, want < 0 ? least : greatest);
    else
      ce = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (ce != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    hipEvent_t ev[5];
    for (int i = 0; i < 5; ++i) {
      if (hipEventCreateWithFlags(&ev[i], side_event_flags()) != hipSuccess) {
        for (int j = 0; j < i; ++j) (void)hipEventDestroy(ev[j]);
        (void)hipStreamDestroy(st);
        (void)hipGetLastError();
        return false;
      }
    }
    ss.s = st;
    ss.fork = ev[0];
    ss.join = ev[1];
    ss.gate = ev[2];
    ss.joinB = ev[3];
    ss.late = ev[4];
  }
  if ((mean_sched() == 2 || mean_sched() == 3) && !ss.s2) {
    // CDX_SIDEB_PRIO: the mean chunks' stream priority (0 normal, default: the merge's workgroups are
    // dispatched first and the mean fills the CUs around them; > 0 highest, < 0 lowest)
    const char* pe = cdx::ab_env("CDX_SIDEB_PRIO");
    const int want = pe ? atoi(pe) : 0;
    int least = 0, greatest = 0;
    hipStream_t st;
    hipError_t ce;
    if (want != 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      ce = hipStreamCreateWithPriority(&st, hipStreamNonBlocking, want < 0 ? least : greatest);
    else
      ce = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipEvent_t ev[4];
    int made = 0;
    if (ce == hipSuccess)
      for (; made < 4; ++made)
        if (hipEventCreateWithFlags(&ev[made], side_event_flags()) != hipSuccess) break;
    if (ce != hipSuccess || made < 4) {
      for (int j = 0; j < made; ++j) (void)hipEventDestroy(ev[j]);
      if (ce == hipSuccess) (void)hipStreamDestroy(st);
      (void)hipGetLastError();
      return false;
    }
    ss.s2 = st;
    ss.g1 = ev[0];
    ss.g2 = ev[1];
    ss.e2a = ev[2];
    ss.jb = ev[3];
  }
  out = ss;
  return true;
}

bool problem_ok(const cdx_problem* p) {
  if (!p || !chain_ok(&p->chain)) return false;
  if (p->n_levels < 1 || p->n_levels > CDX_MAX_LEVELS) return false;
  if (p->n_query_levels < 1 || p->n_query_levels > p->n_levels) return false;
  for (int k = 0; k < p->n_levels; ++k)
    if (p->level_query[k] < 0 || p->level_query[k] >= p->n_query_levels) return false;
  return true;
}

// The level kernel (per (level, candidate)) and the combine kernel (per candidate and fingertip) of a
// closure, dispatched on the fingertip count, gravity, Kabsch records (krot) and chain depth.
template <bool VL>
int launch_level(const cdx_problem* p, int64_t E, const double* q, const double* comp, const double* target,
                 const double* kabsch_noise, uint64_t seed, const ClosureWs& w, const GpisView& gv, int32_t* flip,
                 const double* krot, hipStream_t s) {
  const int64_t KE = (int64_t)p->n_levels * E;
  const dim3 lgrid((unsigned)((KE + 63) / 64));
  if (p->chain.n_tips == 4 && p->gravity && krot)
    hipLaunchKernelGGL((closure_level_kernel<4, 1, true, VL>), lgrid, dim3(64), 0, s, *p, E, q, comp, target, w.X,
                       kabsch_noise, seed, gv, w.lvl, flip, krot);
  else if (p->chain.n_tips == 4 && p->gravity)
    hipLaunchKernelGGL((closure_level_kernel<4, 1, false, VL>), lgrid, dim3(64), 0, s, *p, E, q, comp, target, w.X,
                       kabsch_noise, seed, gv, w.lvl, flip, krot);
  else if (p->chain.n_tips == 4)
    hipLaunchKernelGGL((closure_level_kernel<4, 0, false, VL>), lgrid, dim3(64), 0, s, *p, E, q, comp, target, w.X,
                       kabsch_noise, seed, gv, w.lvl, flip, krot);
  else
    hipLaunchKernelGGL((closure_level_kernel<0, -1, false, VL>), lgrid, dim3(64), 0, s, *p, E, q, comp, target, w.X,
                       kabsch_noise, seed, gv, w.lvl, flip, krot);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

template <bool VL>
int launch_combine(const cdx_problem* p, int64_t E, const double* q, const double* palm_pos, const double* palm_ori,
                   const GpisView& gv, const ClosureWs& w, double* total_loss, double* total_margin, double* g_q,
                   double* g_comp, double* g_target, double* g_palm_pos, double* g_palm_ori, hipStream_t s) {
  const bool sh = shallow_chain(p->chain);
  const dim3 cb(COMBINE_BLOCK);
  if (p->chain.n_tips <= 4) {
    const dim3 cg((unsigned)((E * 4 + COMBINE_BLOCK - 1) / COMBINE_BLOCK));
    if (sh)
      hipLaunchKernelGGL((closure_combine_kernel<4, 8, VL>), cg, cb, 0, s, *p, E, q, palm_pos, palm_ori, gv, w.lvl,
                         total_loss, total_margin, g_q, g_comp, g_target, g_palm_pos, g_palm_ori);
    else
      hipLaunchKernelGGL((closure_combine_kernel<4, CDX_MAX_DEPTH, VL>), cg, cb, 0, s, *p, E, q, palm_pos, palm_ori, gv,
                         w.lvl, total_loss, total_margin, g_q, g_comp, g_target, g_palm_pos, g_palm_ori);
  } else {
    const dim3 cg((unsigned)((E * 8 + COMBINE_BLOCK - 1) / COMBINE_BLOCK));
    if (sh)
      hipLaunchKernelGGL((closure_combine_kernel<8, 8, VL>), cg, cb, 0, s, *p, E, q, palm_pos, palm_ori, gv, w.lvl,
                         total_loss, total_margin, g_q, g_comp, g_target, g_palm_pos, g_palm_ori);
    else
      hipLaunchKernelGGL((closure_combine_kernel<8, CDX_MAX_DEPTH, VL>), cg, cb, 0, s, *p, E, q, palm_pos, palm_ori, gv,
                         w.lvl, total_loss, total_margin, g_q, g_comp, g_target, g_palm_pos, g_palm_ori);
  }
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

// Test hook (cdx_debug_fail_next_closure): the next screened closure returns CDX_ELAUNCH at injection
// point `stage` (1: after the screen / selection and the side-stream fork, 2: after the exact pass,
// 3: after the ∇std pass), through the same error path as a failed launch — one-shot.
std::atomic<int> g_fail_stage{0};
bool inject_fail(int stage) {
  int want = stage;
  return g_fail_stage.load(std::memory_order_relaxed) == stage &&
         g_fail_stage.compare_exchange_strong(want, 0, std::memory_order_relaxed);
}

// The screened closure's repair pass (CDX_SCREEN_REPAIR, default 1; 0 only for the cost A/B): when any
// check of the closure failed — a kept or audited estimate off by more than its margin, an audited row
// that is its group's exact maximum, a maximum on an unrun row — every all-tip row runs the exact pass
// and the groups select as the unscreened closure does, inside the same closure (gated launches: no
// host sync, hipGraph-capturable).
bool screen_repair() {
  static const bool on = [] {
    const char* e = cdx::ab_env("CDX_SCREEN_REPAIR");
    return !e || atoi(e) != 0;
  }();
  return on;
}

// The variance cost added by the combine kernel instead of the level kernel (CDX_VAR_LATE, default 1; 0 for
// the A/B): the level kernel then reads no std, and the screened closure with the forked mean runs it on the
// side stream right after the mean — beside the merge / exact selection / ∇std passes instead of after them.
bool var_late() {
  static const bool on = [] {
    const char* e = getenv("CDX_VAR_LATE");
    return !e || atoi(e) != 0;
  }();
  return on;
}

}  // namespace

extern "C" {

int cdx_fk_forward(const cdx_chain* chain, const float* q, int64_t B, float* pos, float* quat, cdx_stream_t stream) {
  if (!chain_ok(chain)) return CDX_ECHAIN;
  if (B < 0 || (B > 0 && (!q || !pos))) return CDX_EINVAL;
  if (B == 0) return CDX_OK;
  hipLaunchKernelGGL(fk_forward_kernel, dim3((unsigned)((B * chain->n_tips + 63) / 64)), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), *chain, q, B, pos, quat);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_fk_backward(const cdx_chain* chain, const float* q, int64_t B, const float* grad_pos, float* grad_q,
                    cdx_stream_t stream) {
  if (!chain_ok(chain)) return CDX_ECHAIN;
  if (B < 0 || (B > 0 && (!q || !grad_pos || !grad_q))) return CDX_EINVAL;
  if (B == 0) return CDX_OK;
  if (shallow_chain(*chain))
    hipLaunchKernelGGL(fk_backward_kernel<8>, dim3((unsigned)((B + 63) / 64)), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), *chain, q, B, grad_pos, grad_q);
  else
    hipLaunchKernelGGL(fk_backward_kernel<CDX_MAX_DEPTH>, dim3((unsigned)((B + 63) / 64)), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), *chain, q, B, grad_pos, grad_q);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_force_eq_forward(const cdx_force_eq* p, int64_t B, const double* tip, const double* target, const double* comp,
                         const double* normal, const double* noise, uint64_t seed, double* reward, double* margin,
                         double* force_norm, int32_t* flip, cdx_stream_t stream) {
  if (!p || p->n_tips < 1 || p->n_tips > CDX_MAX_TIPS || B < 0) return CDX_EINVAL;
  if (B == 0) return CDX_OK;
  if (!tip || !target || !comp || !normal || !reward || !margin || !force_norm) return CDX_EINVAL;
  const dim3 grid((unsigned)((B + 63) / 64));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (p->n_tips == 4)
    hipLaunchKernelGGL(force_eq_forward_kernel<4>, grid, dim3(64), 0, s, *p, B, tip, target, comp, normal, noise, seed,
                       reward, margin, force_norm, flip);
  else
    hipLaunchKernelGGL(force_eq_forward_kernel<0>, grid, dim3(64), 0, s, *p, B, tip, target, comp, normal,
                       noise, seed, reward, margin, force_norm, flip);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_force_eq_backward(const cdx_force_eq* p, int64_t B, const double* tip, const double* target, const double* comp,
                          const double* normal, const double* noise, uint64_t seed, const double* g_reward,
                          const double* g_force_norm, double* g_tip, double* g_target, double* g_comp,
                          cdx_stream_t stream) {
  if (!p || p->n_tips < 1 || p->n_tips > CDX_MAX_TIPS || B < 0) return CDX_EINVAL;
  if (B == 0) return CDX_OK;
  if (!tip || !target || !comp || !normal || !g_tip || !g_target || !g_comp) return CDX_EINVAL;
  const dim3 grid((unsigned)((B + 63) / 64));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (p->n_tips == 4)
    hipLaunchKernelGGL(force_eq_backward_kernel<4>, grid, dim3(64), 0, s, *p, B, tip, target, comp, normal, noise, seed,
                       g_reward, g_force_norm, g_tip, g_target, g_comp);
  else
    hipLaunchKernelGGL(force_eq_backward_kernel<0>, grid, dim3(64), 0, s, *p, B, tip, target, comp, normal,
                       noise, seed, g_reward, g_force_norm, g_tip, g_target, g_comp);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_collision_loss(const cdx_collision* c, int64_t E, const double* q, const double* palm_pos,
                       const double* palm_ori, double* cost, double* g_q, double* g_palm_pos, double* g_palm_ori,
                       int32_t accumulate, cdx_stream_t stream) {
  if (!c || !chain_ok(&c->chain)) return CDX_ECHAIN;
  if (c->n_pairs < 0 || c->n_pairs > CDX_MAX_PAIRS) return CDX_EINVAL;
  for (int p = 0; p < c->n_pairs; ++p)
    for (int j = 0; j < 2; ++j)
      if (c->pairs[p][j] < 0 || c->pairs[p][j] >= c->chain.n_tips) return CDX_EINVAL;
  if (E < 0 || (E > 0 && (!q || !palm_pos || !palm_ori || !cost || !g_q || !g_palm_pos || !g_palm_ori)))
    return CDX_EINVAL;
  if (E == 0) return CDX_OK;
  hipLaunchKernelGGL(collision_kernel, dim3((unsigned)((E + 63) / 64)), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), *c, E, q, palm_pos, palm_ori, cost, g_q, g_palm_pos,
                     g_palm_ori, accumulate);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

size_t cdx_closure_workspace(const cdx_problem* p, int64_t E) {
  if (!problem_ok(p) || E <= 0) return 0;
  return closure_ws_layout(p, E, nullptr).bytes;
}

int cdx_closure(const cdx_problem* p, int64_t E, const double* q, const double* comp, const double* target,
                const double* palm_pos, const double* palm_ori, const double* kabsch_noise, uint64_t seed,
                void* workspace, double* total_loss, double* total_margin, double* pregrasp_tip, double* g_q,
                double* g_comp, double* g_target, double* g_palm_pos, double* g_palm_ori, int32_t* flip,
                cdx_stream_t stream) {
  if (!problem_ok(p)) return CDX_EINVAL;
  if (E < 0) return CDX_EINVAL;
  if (E == 0) return CDX_OK;
  if (!q || !comp || !target || !palm_pos || !palm_ori || !workspace || !total_loss || !total_margin || !g_q ||
      !g_comp || !g_target || !g_palm_pos || !g_palm_ori)
    return CDX_EINVAL;
  if (!p->gpis.Ainv || !p->gpis.Linv_t || !p->gpis.Linv || !p->gpis.X1 || !p->gpis.alpha) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  ClosureWs w = closure_ws_layout(p, E, static_cast<char*>(workspace));
  const int64_t Mq = cdx::n_queries(*p, E);
  const int64_t Ms = (int64_t)p->n_query_levels * E * p->chain.n_tips;
  const dim3 grid((unsigned)((E * p->chain.n_tips + 63) / 64));
  cdx::prof_mark(cdx::PROF_QUERIES, true, s);
  hipLaunchKernelGGL(closure_queries_kernel, grid, dim3(64), 0, s, *p, E, q, target, palm_pos, palm_ori, w.X,
                     pregrasp_tip);
  cdx::prof_mark(cdx::PROF_QUERIES, false, s);
  if (hipGetLastError() != hipSuccess) return CDX_ELAUNCH;
  const bool scr = screen_on(p, E);
  SideStream ss;
  const bool fork = scr && fork_mean() && side_stream(ss);
  const SideStream* pending_b = nullptr;  // mean B still to be joined before the combine kernel
  const double* krot = nullptr;           // Kabsch records computed ahead (else the level kernel's own SVD)
  cdx::GradFold fold;                      // ∇std finalize folded into the level (or combine) kernel (screened)
  const bool vlate = var_late();
  bool level_early = false;                // the level kernel already queued (side stream, after the mean)
  int rc;
  if (!fork) {
    rc = cdx_gpis_mean(&p->gpis, w.X, Mq, w.mean, w.gmean, w.normal, stream);
    if (rc) return rc;
  }
  // whitened std at every all-tip query, keeping V = (L⁻¹K*ᵀ)ᵀ for the ∇std pass
  // … and the ∇std fingertip of each (distinct level, candidate): the all-tip rows q_alltip(u, e, f)
  // = (u·E + e)·T + f form groups of T, selected in the std finalize
  const int64_t Mg = (int64_t)p->n_query_levels * E;
  if (scr) {
    // bf16 screen of every all-tip row → exact whitened fp64 pass for the fingertips that can still
    // be their group's maximum (≈ 1 per group) → ∇std at the group's maximum from its kept V row;
    // the mean on the side stream beside the screen (SideStream)
    const int T = p->chain.n_tips;
    // Once the fork point has passed, every return joins the side stream back into `s` first:
    // under capture an unjoined fork invalidates the graph, and eagerly the mean would keep writing
    // the workspace after the error return.  (A join recorded before a failed launch_fork only waits
    // on the event's previous record.)
    bool forked = false, forkedB = false;
    const int64_t MqA = mean_split() ? (int64_t)(p->n_query_levels + 1) * E * T : Mq;  // rows of mean A
    const cdx_stream_t side = reinterpret_cast<cdx_stream_t>(ss.s);
    // The Kabsch records (closure_kabsch_kernel, kabsch_mode() 1): first on the side stream, right
    // after the screen kernel (the screen's waves leave too few registers for them to run beside it;
    // after it they share the chip with the latency-bound selection and compaction), then mean A on
    // the same stream — one fork, one join: every event record / wait on `s` costs ≈ 5 µs of stream
    // time (profiles/r03s_*).  The mean is effectively serial after the refine pass anyway (it cannot
    // share a CU with it), so queueing it behind the records costs nothing.
    const int kmode = fork ? kabsch_mode() : 0;
    auto launch_records = [&](hipStream_t st) {
      const int64_t KE = (int64_t)p->n_levels * E;
      const dim3 kg((unsigned)((KE + 63) / 64));
      if (T == 4 && p->gravity)
        hipLaunchKernelGGL((closure_kabsch_kernel<4, 1>), kg, dim3(64), 0, st, *p, E, comp, target, w.X, kabsch_noise,
                           seed, w.krot);
      else if (T == 4)
        hipLaunchKernelGGL((closure_kabsch_kernel<4, 0>), kg, dim3(64), 0, st, *p, E, comp, target, w.X, kabsch_noise,
                           seed, w.krot);
      else
        hipLaunchKernelGGL((closure_kabsch_kernel<0, -1>), kg, dim3(64), 0, st, *p, E, comp, target, w.X,
                           kabsch_noise, seed, w.krot);
      return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
    };
    // mean_sched 4: the fork runs the records only; launch_late queues the mean and the level kernel behind
    // the refine kernel's event
    const bool late = kmode == 1 && vlate && !mean_split() && !mean_first() && mean_sched() == 4;
    auto launch_fork = [&]() -> int {
      forked = true;
      if (hipEventRecord(ss.fork, s) != hipSuccess || hipStreamWaitEvent(ss.s, ss.fork, 0) != hipSuccess) return CDX_ELAUNCH;
      if (kmode == 1 && !mean_first()) {
        const int r = launch_records(ss.s);
        if (r) return r;
      }
      if (late) return hipEventRecord(ss.join, ss.s) != hipSuccess ? CDX_ELAUNCH : CDX_OK;
      int r = cdx_gpis_mean(&p->gpis, w.X, MqA, w.mean, w.gmean, w.normal, side);
      if (r) return r;
      if (kmode == 1 && mean_first() && (r = launch_records(ss.s))) return r;
      if (vlate) {  // the level kernel reads the mean A rows, the Kabsch records and no std
        GpisView gv0;
        gv0.mean = w.mean; gv0.gmean = w.gmean; gv0.normal = w.normal; gv0.std_ = w.std_; gv0.gstd = w.gstd;
        gv0.E = E; gv0.T = T; gv0.Lq = p->n_query_levels; gv0.e = 0;
        r = launch_level<true>(p, E, q, comp, target, kabsch_noise, seed, w, gv0, flip, kmode == 1 ? w.krot : nullptr,
                               ss.s);
        if (r) return r;
        level_early = true;
      }
      return hipEventRecord(ss.join, ss.s) != hipSuccess ? CDX_ELAUNCH : CDX_OK;
    };
    auto launch_late = [&]() -> int {  // after the main stream recorded ss.late
      if (hipStreamWaitEvent(ss.s, ss.late, 0) != hipSuccess) return CDX_ELAUNCH;
      int r = cdx_gpis_mean(&p->gpis, w.X, Mq, w.mean, w.gmean, w.normal, side);
      if (r) return r;
      GpisView gv0;
      gv0.mean = w.mean; gv0.gmean = w.gmean; gv0.normal = w.normal; gv0.std_ = w.std_; gv0.gstd = w.gstd;
      gv0.E = E; gv0.T = T; gv0.Lq = p->n_query_levels; gv0.e = 0;
      r = launch_level<true>(p, E, q, comp, target, kabsch_noise, seed, w, gv0, flip, w.krot, ss.s);
      if (r) return r;
      level_early = true;
      return hipEventRecord(ss.join, ss.s) != hipSuccess ? CDX_ELAUNCH : CDX_OK;
    };
    auto launch_b = [&]() -> int {  // mean B, gated behind the work already on `s`
      if (MqA >= Mq) return CDX_OK;
      forkedB = true;
      if (hipEventRecord(ss.gate, s) != hipSuccess || hipStreamWaitEvent(ss.s, ss.gate, 0) != hipSuccess) return CDX_ELAUNCH;
      const int r = cdx_gpis_mean(&p->gpis, w.X + 3 * MqA, Mq - MqA, w.mean + MqA, w.gmean + 3 * MqA,
                                  w.normal + 3 * MqA, side);
      if (r) return r;
      return hipEventRecord(ss.joinB, ss.s) != hipSuccess ? CDX_ELAUNCH : CDX_OK;
    };
    // The split mean schedule (mean_sched 2; needs the records ahead, the variance cost in the combine and
    // no mean A/B split): side A = ss.s runs the Kabsch records and the level kernel, side B = ss.s2 the
    // mean chunks.  Phase 1 at the fork point: A records; B rows [0, M1), then g1 (the refine pass waits
    // for it).  Phase 2 right after the refine kernel (g2 recorded between it and the merge): B the
    // remaining all-tip / target rows, e2a, the pregrasp / palm rows; A waits e2a, runs the level kernel and
    // records join; B waits join and records jb, which the main stream waits for before the combine.
    const bool sched2 = fork && kabsch_mode() == 1 && vlate && !mean_split() && (mean_sched() == 2 || mean_sched() == 3) && ss.s2;
    // 3: the ∇std pass waits for both side streams (mean chunks, level kernel) instead of the combine, so
    // that no mean / level workgroup holds a CU the pass needs
    const bool wait_before_grad = sched2 && mean_sched() == 3;
    bool joined_early = false;
    const int64_t M01 = (int64_t)(p->n_query_levels + 1) * E * T;  // all-tip + target rows (the level kernel's)
    const int64_t M1 = sched2 ? std::min<int64_t>(Mq, (int64_t)(mean_chunk1() * (double)Mq)) : 0;
    bool forked2 = false;
    const cdx_stream_t sideB = reinterpret_cast<cdx_stream_t>(ss.s2);
    auto mean_rows = [&](int64_t a, int64_t b, cdx_stream_t st) -> int {
      if (b <= a) return CDX_OK;
      return cdx_gpis_mean(&p->gpis, w.X + 3 * a, b - a, w.mean + a, w.gmean + 3 * a, w.normal + 3 * a, st);
    };
    auto launch_fork2 = [&]() -> int {
      forked = forked2 = true;
      if (hipEventRecord(ss.fork, s) != hipSuccess || hipStreamWaitEvent(ss.s, ss.fork, 0) != hipSuccess ||
          hipStreamWaitEvent(ss.s2, ss.fork, 0) != hipSuccess)
        return CDX_ELAUNCH;
      int r = launch_records(ss.s);
      if (!r) r = mean_rows(0, M1, sideB);
      if (!r && hipEventRecord(ss.g1, ss.s2) != hipSuccess) r = CDX_ELAUNCH;
      return r;
    };
    auto launch_phase2 = [&]() -> int {  // after the main stream recorded g2
      if (hipStreamWaitEvent(ss.s2, ss.g2, 0) != hipSuccess) return CDX_ELAUNCH;
      int r = mean_rows(M1, std::max(M1, M01), sideB);
      if (!r && hipEventRecord(ss.e2a, ss.s2) != hipSuccess) r = CDX_ELAUNCH;
      if (!r) r = mean_rows(std::max(M1, M01), Mq, sideB);
      if (r) return r;
      if (hipStreamWaitEvent(ss.s, ss.e2a, 0) != hipSuccess) return CDX_ELAUNCH;
      GpisView gv0;
      gv0.mean = w.mean; gv0.gmean = w.gmean; gv0.normal = w.normal; gv0.std_ = w.std_; gv0.gstd = w.gstd;
      gv0.E = E; gv0.T = T; gv0.Lq = p->n_query_levels; gv0.e = 0;
      r = launch_level<true>(p, E, q, comp, target, kabsch_noise, seed, w, gv0, flip, w.krot, ss.s);
      if (r) return r;
      level_early = true;
      if (hipEventRecord(ss.join, ss.s) != hipSuccess || hipStreamWaitEvent(ss.s2, ss.join, 0) != hipSuccess ||
          hipEventRecord(ss.jb, ss.s2) != hipSuccess)
        return CDX_ELAUNCH;
      return CDX_OK;
    };
    auto joined = [&](int r) -> int {
      if (forked2) {  // both side streams' queued work, whichever phase failed
        if ((hipEventRecord(ss.join, ss.s) != hipSuccess || hipEventRecord(ss.jb, ss.s2) != hipSuccess ||
             hipStreamWaitEvent(s, ss.join, 0) != hipSuccess || hipStreamWaitEvent(s, ss.jb, 0) != hipSuccess) && !r)
          r = CDX_ELAUNCH;
        return r;
      }
      if (forked && hipStreamWaitEvent(s, ss.join, 0) != hipSuccess && !r) r = CDX_ELAUNCH;
      if (forkedB && hipStreamWaitEvent(s, ss.joinB, 0) != hipSuccess && !r) r = CDX_ELAUNCH;
      return r;
    };
    // the mean's fork point (kabsch_mode 1 forks once, after the screen, whatever fork_point says)
    const int fp = kmode == 1 ? 4 : (fork ? fork_point() : 0);
    if (fp == 1 && (rc = launch_fork())) return joined(rc);
    auto fork_cb = [](void* c) { return (*static_cast<decltype(launch_fork)*>(c))(); };
    auto fork2_cb = [](void* c) { return (*static_cast<decltype(launch_fork2)*>(c))(); };
    rc = sched2 ? cdx::screen_select_launch(p->gpis, w.X, Mg, T, w.screen_ws, w.sv2, w.std_, w.vpos, w.rows, w.keep,
                                            w.zkey, w.stats, s, +fork2_cb, &launch_fork2)
                : cdx::screen_select_launch(p->gpis, w.X, Mg, T, w.screen_ws, w.sv2, w.std_, w.vpos, w.rows, w.keep,
                                            w.zkey, w.stats, s, fp == 4 ? +fork_cb : nullptr, &launch_fork);
    if (!rc && inject_fail(1)) rc = CDX_ELAUNCH;
    if (rc) return joined(rc);
    if (!sched2 && fp == 2 && (rc = launch_fork())) return joined(rc);
    if (sched2 && hipStreamWaitEvent(s, ss.g1, 0) != hipSuccess) return joined(CDX_ELAUNCH);
    double* rpart = nullptr;
    int64_t rpad = 0;
    rc = cdx::gpis_refine_launch(p->gpis, w.X, w.rows, w.stats + cdx::SS_EXTRA, (int)Mg, Ms, w.refine_ws, w.V, s, &rpart,
                                 &rpad, nullptr, true, sched2 ? ss.g2 : (late && forked ? ss.late : nullptr));
    if (!rc && sched2) rc = launch_phase2();
    if (!rc && late && forked) rc = launch_late();
    if (!rc && inject_fail(2)) rc = CDX_ELAUNCH;
    if (rc) return joined(rc);
    if (!sched2 && fp == 3 && (rc = launch_fork())) return joined(rc);
    rc = cdx::refine_select_launch(p->gpis, w.X, Mg, T, rpart, rpad, w.sv2, w.vpos, w.keep, w.std_, w.var, w.sel,
                                   w.Xg, w.vrow, w.stats, s);
    if (rc) return joined(rc);
    if (screen_repair()) {
      // the repair pass, gated on this closure's checks (a no-op launch pair otherwise): every all-tip row
      // through the exact pass (identity list) and the unscreened selection — no screened result that
      // failed a check leaves the closure, whichever entry point called it
      cdx::RepairSel rs;
      rs.X = w.X; rs.G = Mg; rs.T = T; rs.std_ = w.std_; rs.var = w.var; rs.Xg = w.Xg; rs.sel = w.sel; rs.vrow = w.vrow;
      rs.stats = w.stats;
      rc = cdx::gpis_refine_launch(p->gpis, w.X, nullptr, nullptr, (int)Ms, Ms, w.refine_ws, w.V, s, nullptr, nullptr,
                                   w.stats, false, nullptr, &rs);
      if (rc) return joined(rc);
    }
    if (wait_before_grad) {
      if (hipStreamWaitEvent(s, ss.jb, 0) != hipSuccess) return joined(CDX_ELAUNCH);
      joined_early = true;
    } else if (forked && !sched2 && !forkedB && join_early()) {
      if (hipStreamWaitEvent(s, ss.join, 0) != hipSuccess) return joined(CDX_ELAUNCH);
      joined_early = true;
    }
    rc = cdx::gpis_grad_launch(p->gpis, w.Xg, Mg, w.sel, w.var, w.gstd, w.grad_ws, s, w.V, w.vrow,
                               grad_fold() ? &fold : nullptr);
    if (!rc && inject_fail(3)) rc = CDX_ELAUNCH;
    if (rc) return joined(rc);
    if (fork && !sched2 && (rc = launch_b())) return joined(rc);
    // mean A (and the Kabsch records of mode 1) before the level kernel; mean B is joined before the
    // combine kernel below (sched2: jb follows both side streams)
    if (forked && !joined_early && hipStreamWaitEvent(s, sched2 ? ss.jb : ss.join, 0) != hipSuccess) {
      forked = forked2 = false;
      return joined(CDX_ELAUNCH);
    }
    if (kmode == 1 && forked) krot = w.krot;
    if (forkedB) pending_b = &ss;
  } else {
    const cdx::VarSelect vs{p->chain.n_tips, w.sel, w.Xg};
    rc = cdx::gpis_var_launch(p->gpis, w.X, Ms, w.std_, w.var, w.var_ws, s, w.V, &vs);
    if (rc) return rc;
    rc = cdx::gpis_grad_launch(p->gpis, w.Xg, Mg, w.sel, w.var, w.gstd, w.grad_ws, s, w.V);
  }
  if (rc) return rc;
  GpisView gv;
  gv.mean = w.mean; gv.gmean = w.gmean; gv.normal = w.normal; gv.std_ = w.std_; gv.gstd = w.gstd;
  gv.E = E; gv.T = p->chain.n_tips; gv.Lq = p->n_query_levels; gv.e = 0;
  GpisView gvl = gv;  // ∇std from the pass's pieces when folded (the level kernel's view, or the combine's: vlate)
  gvl.fold = fold;
  gvl.var = w.var;
  gvl.sel = w.sel;
  cdx::prof_mark(cdx::PROF_COST, true, s);
  if (!level_early) {
    rc = vlate ? launch_level<true>(p, E, q, comp, target, kabsch_noise, seed, w, gv, flip, krot, s)
               : launch_level<false>(p, E, q, comp, target, kabsch_noise, seed, w, gvl, flip, krot, s);
    if (rc) {
      if (pending_b) (void)hipStreamWaitEvent(s, pending_b->joinB, 0);
      return rc;
    }
  }
  if (pending_b && hipStreamWaitEvent(s, pending_b->joinB, 0) != hipSuccess) return CDX_ELAUNCH;
  rc = vlate ? launch_combine<true>(p, E, q, palm_pos, palm_ori, gvl, w, total_loss, total_margin, g_q, g_comp, g_target,
                                    g_palm_pos, g_palm_ori, s)
             : launch_combine<false>(p, E, q, palm_pos, palm_ori, gv, w, total_loss, total_margin, g_q, g_comp, g_target,
                                     g_palm_pos, g_palm_ori, s);
  if (rc) return rc;
  cdx::prof_mark(cdx::PROF_COST, false, s);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_ab_switches(void) {
#if defined(CDX_AB_SWITCHES)
  return 1;
#else
  return 0;
#endif
}

int cdx_debug_fail_next_closure(int32_t stage) {
  if (stage < 0 || stage > 3) return CDX_EINVAL;
  g_fail_stage.store(stage, std::memory_order_relaxed);
  return CDX_OK;
}

int cdx_closure_screen_stats(const cdx_problem* p, int64_t E, const void* workspace, int32_t* out) {
  if (!problem_ok(p) || E <= 0 || !workspace || !out) return CDX_EINVAL;
  if (!screen_on(p, E)) {
    out[0] = out[1] = out[2] = -1;
    return CDX_OK;
  }
  ClosureWs w = closure_ws_layout(p, E, static_cast<char*>(const_cast<void*>(workspace)));
  int st[2] = {0, 0};
  if (hipMemcpy(st, w.stats, sizeof(st), hipMemcpyDeviceToHost) != hipSuccess) return CDX_ELAUNCH;
  out[0] = (int32_t)((int64_t)p->n_query_levels * E + st[cdx::SS_EXTRA]);  // rows of the exact pass
  out[1] = st[cdx::SS_MISS];                                                // estimates off by more than Δ
  out[2] = (int32_t)((int64_t)p->n_query_levels * E * p->chain.n_tips);     // all-tip rows screened
  return CDX_OK;
}

int cdx_closure_screen_report(const cdx_problem* p, int64_t E, const void* workspace, cdx_screen_report* out,
                              cdx_stream_t stream) {
  if (!problem_ok(p) || E <= 0 || !workspace || !out) return CDX_EINVAL;
  *out = cdx_screen_report{};
  if (!screen_on(p, E)) return CDX_OK;
  ClosureWs w = closure_ws_layout(p, E, static_cast<char*>(const_cast<void*>(workspace)));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int st[cdx::SS_WORDS];
  if (hipMemcpyAsync(st, w.stats, sizeof(st), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return CDX_ELAUNCH;
  auto ratio = [&](int k) { return (double)__builtin_bit_cast(float, st[k]); };
  const int64_t Mg = (int64_t)p->n_query_levels * E;
  out->screened = 1;
  out->screened_rows = (int32_t)(Mg * p->chain.n_tips);
  out->exact_rows = (int32_t)(Mg + st[cdx::SS_EXTRA]);
  out->audited_rows = st[cdx::SS_AUDIT];
  out->bound_misses = st[cdx::SS_MISS];
  out->audit_misses = st[cdx::SS_AUDIT_MISS];
  out->audit_flips = st[cdx::SS_AUDIT_FLIP];
  out->faults = st[cdx::SS_FAULT];
  out->max_ratio = ratio(cdx::SS_RATIO);
  out->max_ratio_audit = ratio(cdx::SS_RATIO_AUDIT);
  const int c = cdx::SS_CUM;
  out->cum_closures = (uint32_t)st[c];
  out->cum_audited_rows = (uint32_t)st[c + cdx::SS_AUDIT];
  out->cum_bound_misses = (uint32_t)st[c + cdx::SS_MISS];
  out->cum_audit_misses = (uint32_t)st[c + cdx::SS_AUDIT_MISS];
  out->cum_audit_flips = (uint32_t)st[c + cdx::SS_AUDIT_FLIP];
  out->cum_faults = (uint32_t)st[c + cdx::SS_FAULT];
  out->cum_max_ratio = ratio(c + cdx::SS_RATIO);
  out->cum_max_ratio_audit = ratio(c + cdx::SS_RATIO_AUDIT);
  out->repaired = st[cdx::SS_REPAIR];
  out->discarded_rows = st[cdx::SS_DISCARD];
  out->min_gap = ratio(cdx::SS_GAP);
  out->audit_cut = ratio(cdx::SS_AUDIT_CUT);
  out->cum_repairs = (uint32_t)st[c + cdx::SS_REPAIR];
  out->cum_discarded_rows = (uint32_t)st[c + cdx::SS_DISCARD];
  const unsigned cg = (unsigned)st[c + cdx::SS_GAP];  // 0xFFFFFFFF − bits of the smallest gap, 0: none
  out->cum_min_gap = cg ? (double)__builtin_bit_cast(float, 0xFFFFFFFFu - cg) : INFINITY;
  return CDX_OK;
}

int cdx_closure_screen_reset(const cdx_problem* p, int64_t E, void* workspace, cdx_stream_t stream) {
  if (!problem_ok(p) || E < 0) return CDX_EINVAL;
  if (E == 0 || !screen_on(p, E)) return CDX_OK;
  if (!workspace) return CDX_EINVAL;
  ClosureWs w = closure_ws_layout(p, E, static_cast<char*>(workspace));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(w.stats + cdx::SS_CUM, 0, (cdx::SS_WORDS - cdx::SS_CUM) * sizeof(int), s) != hipSuccess)
    return CDX_ELAUNCH;
  const int64_t Ms = (int64_t)p->n_query_levels * E * p->chain.n_tips;
  return cdx::gpis_refine_reset(p->gpis, Ms, w.refine_ws, s);
}

const char* cdx_version(void) { return "compliancedex_amd 0.1 gfx950"; }

}  // extern "C"

namespace cdx {
namespace {
constexpr int PROF_POOL = 4096;
struct Prof {
  unsigned mask = 0;  // stages recorded
  hipEvent_t ev[PROF_STAGES][PROF_POOL][2];
  int n[PROF_STAGES] = {};
  bool created = false;
} g_prof;
}  // namespace

void prof_mark(int stage, bool begin, hipStream_t s) {
  if (!((g_prof.mask >> stage) & 1u)) return;
  const int i = g_prof.n[stage];
  if (i >= PROF_POOL) return;
  (void)hipEventRecord(g_prof.ev[stage][i][begin ? 0 : 1], s);
  if (!begin) g_prof.n[stage] = i + 1;
}
}  // namespace cdx

extern "C" int cdx_profile_enable(int stages) {
  using cdx::g_prof;
  const unsigned on = (unsigned)stages & ((1u << cdx::PROF_STAGES) - 1);
  if (on && !g_prof.created) {
    // timing-only events: no system-scope fence (L2 writeback) at each record; CDX_PROF_EVENT_FLAGS
    // (hex) overrides the flags for A/B runs
    unsigned flags = hipEventDisableSystemFence;
    if (const char* f = cdx::ab_env("CDX_PROF_EVENT_FLAGS")) flags = (unsigned)strtoul(f, nullptr, 16);
    const int total = cdx::PROF_STAGES * cdx::PROF_POOL * 2;
    hipEvent_t* evs = &g_prof.ev[0][0][0];
    for (int e = 0; e < total; ++e)
      if (hipEventCreateWithFlags(&evs[e], flags) != hipSuccess) {
        (void)hipGetLastError();  // not left pending for the caller's next launch check
        for (int k = 0; k < e; ++k) (void)hipEventDestroy(evs[k]);  // no partial pool is kept
        return CDX_EINVAL;
      }
    g_prof.created = true;
  }
  g_prof.mask = on;
  for (int st = 0; st < cdx::PROF_STAGES; ++st) g_prof.n[st] = 0;
  return CDX_OK;
}

// Sums the recorded kernel times per stage (ms) and launch counts, then resets the pool.
extern "C" int cdx_profile_read(double* ms, int64_t* count) {
  using cdx::g_prof;
  for (int st = 0; st < cdx::PROF_STAGES; ++st) {
    double tot = 0;
    for (int i = 0; i < g_prof.n[st]; ++i) {
      if (hipEventSynchronize(g_prof.ev[st][i][1]) != hipSuccess) return CDX_ELAUNCH;
      float t = 0;
      if (hipEventElapsedTime(&t, g_prof.ev[st][i][0], g_prof.ev[st][i][1]) != hipSuccess) return CDX_ELAUNCH;
      tot += t;
    }
    ms[st] = tot;
    count[st] = g_prof.n[st];
    g_prof.n[st] = 0;
  }
  return CDX_OK;
}

extern "C" void cdx_abi_sizes(size_t* out) {
  out[0] = sizeof(cdx_gpis);
  out[1] = sizeof(cdx_body);
  out[2] = sizeof(cdx_chain);
  out[3] = sizeof(cdx_problem);
  out[4] = sizeof(cdx_collision);
  out[5] = sizeof(cdx_adam);
  out[6] = sizeof(cdx_opt_buffers);
  out[7] = sizeof(cdx_force_eq);
  out[8] = sizeof(cdx_screen_report);
  out[9] = sizeof(cdx_kin_params);
  out[10] = sizeof(cdx_kin_opt);
  out[11] = sizeof(cdx_kin_opt_buffers);
  out[12] = sizeof(cdx_sdf_batch_query);
}
