// Kin-mode (KinGraspOptimizer, optimize_pregrasp.py:121-227) cost assembly and backward for gfx950: one
// lane per candidate takes the iteration's fingertips (FK + palm offset), the three TorchSDF queries'
// outputs and the parameters, and returns the loss l, the force-closure margins, the blended contact
// normals and the gradients of l w.r.t. the joint angles, targets and compliances — the reference's
// ~30 elementwise ops, its force_eq_reward and the autograd backward through them, TorchSDF and the FK
// chain (:183-208), in one launch.
//
//   normal_f   = normalize(½·s1_f·n1_f + ½·s2_f·n2_f)          (tips vs deflated / true mesh, :186-187; f32)
//   l          = −5·reward + 1000·Σ√d_f + 10·Σ ts_f·√td_f + 10·|mean tip − mean target|
//                − Σ clamp(fn_f·softmin(fn)_f, max = 1) + 10·|q − ref_q|          (:195-205)
//   ∂√d/∂tip   = ½/√d · 2(tip − clst)                          (TorchSDF backward, .cu:256-270)
// The per-candidate arithmetic is f64 (the force-equilibrium reward is ForceEq, shared with the closure);
// the normals are formed in f32 as the reference forms them; the FK backward runs in f32 like the
// reference's autograd through compute_forward_kinematics.
#include <hip/hip_runtime.h>

#include "cdx_cost.h"

#pragma clang fp contract(off)

namespace {

#if defined(CDX_KIN_FE_F32)  // (A/B: the reward in the reference's float32 — 0.338 → 0.330 ms per Kin iteration, but its
using FeReal = float;        // SVD backward then divides by S_k² − S_j² = 0 on near-repeated singular values, a NaN the
#else                        // f64 path does not produce there: profiles/r06g_kin_fe_f32_ab.jsonl)
using FeReal = double;
#endif

__device__ __forceinline__ uint64_t kin_mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Joint-angle reader over the workgroup's LDS copy of the candidate's updated row.
struct QRowLds {
  const float* p;
  __device__ __forceinline__ float operator[](int i) const { return p[i]; }
};

// The fused Kin iteration's FK-walk cache (cdx_kin_opt_buffers::fk_state): per 64-lane workgroup a block of FKS_BLOCK
// floats holding, per lane, the final pose R (slots 0–8) and t (9–11) of the lane's fingertip chain, each moving joint's
// world axis and origin at path level l (slots 12 + 6·l … 12 + 6·l + 5) and the joint angles the walk read (the lane's
// DOFs f + 4u at slot 12 + 6·MAXD + u) — written by the step's next-fingertip walk, read by the next iteration's FK
// backward when the candidate's joint row still has exactly those bits.  Slot s of lane l at float
// (s / 4)·256 + 4·l + s % 4: 16-byte units in lane order, so that the writer stores one dwordx4 per four slots
// (a dword store per slot cost ≈ 30 k cycles a wave) and the reader's LDS-DMA copies the block as it lies.
constexpr int FKS_PF = CDX_MAX_DOFS / 4;
constexpr int fks_slots(int maxd) { return 12 + 6 * maxd + FKS_PF; }  // the LDS image
// … and behind the image, in memory only, the iteration that wrote the lane's slots + 1 (a tag: the reader at
// iteration s takes the slots only when it is s — a zero-filled buffer never matches), then 3 free slots
constexpr int fks_tag(int maxd) { return fks_slots(maxd); }
constexpr int FKS_BLOCK = (fks_slots(CDX_MAX_DEPTH) + 4) * 64;
__device__ __forceinline__ int fks_at(int slot, int lane) { return (slot >> 2) * 256 + 4 * lane + (slot & 3); }
static_assert(fks_slots(8) % 4 == 0 && fks_slots(CDX_MAX_DEPTH) % 4 == 0, "whole 1-KB DMA units per block");

#if defined(CDX_KIN_DIAG_PHASES)  // (timing-only diagnostic build: per-wave shader-clock stamps at the kernel's phases)
__device__ unsigned long long g_kin_phase[4096][16];
#define KIN_PHASE(i)                                                                                      \
  do {                                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                           \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_kin_phase[blockIdx.x][i] = t_;                          \
    __builtin_amdgcn_sched_barrier(0);                                                                    \
  } while (0)
#else
#define KIN_PHASE(i) do {} while (0)
#endif

__device__ __forceinline__ float adam_f32(float p, float g, float& m, float& v, float w1, float b2, float w2, float bc2s,
                                          float eps, float step) {
  // torch.optim.Adam's single-tensor / foreach update in float32 opmath: m.lerp_(g, 1 − β1);
  // v.mul_(β2).addcmul_(g, g, 1 − β2); p.addcdiv_(m, sqrt(v)/sqrt(bc2) + eps, −lr/bc1)
  m = m + w1 * (g - m);
  v = v * b2 + (w2 * g) * g;
  const float denom = sqrtf(v) / bc2s + eps;
  return p + step * (m / denom);
}

__device__ __forceinline__ float rmsprop_f32(float p, float g, float& v, float a, float w2, float eps, float lr) {
  // torch.optim.RMSprop (no momentum, not centred): v.mul_(α).addcmul_(g, g, 1 − α); p.addcdiv_(g, sqrt(v) + eps, −lr)
  v = v * a + (w2 * g) * g;
  const float avg = sqrtf(v) + eps;
  return p + lr * (g / avg);
}

// Adam's per-iteration constants (torch.optim.Adam, step count s + 1): 1 − β1, β2, 1 − β2, √(1 − β2^t) and the
// −lr/(1 − β1^t) step sizes of the three groups, as cdx_kin_step and the fused iteration both take them.
struct AdamConst {
  float w1, b2, w2, bc2s, eps, sz[3];
};
__device__ __forceinline__ AdamConst adam_const(const cdx_kin_opt& cfg, int s) {
  const double step = (double)(s + 1);
  const double bc1 = 1.0 - pow(cfg.beta1, step), bc2 = 1.0 - pow(cfg.beta2, step);
  AdamConst a;
  a.w1 = (float)(1.0 - cfg.beta1);
  a.b2 = (float)cfg.beta2;
  a.w2 = (float)(1.0 - cfg.beta2);
  a.bc2s = (float)sqrt(bc2);
  a.eps = (float)cfg.eps;
  for (int g = 0; g < 3; ++g) a.sz[g] = (float)(-(cfg.lr[g] / bc1));
  return a;
}

template <int NT, int MAXD, bool FK>
__global__ __launch_bounds__(64) void kin_cost_kernel(
    cdx_chain chain, cdx_kin_params p, int64_t E, const float* __restrict__ q, const float* __restrict__ tip,
    const float* __restrict__ target, const float* __restrict__ comp, const int32_t* __restrict__ sign1,
    const float* __restrict__ n1, const float* __restrict__ sqd, const int32_t* __restrict__ sign2,
    const float* __restrict__ n2, const float* __restrict__ clst, const float* __restrict__ tsqd,
    const int32_t* __restrict__ tsign, const float* __restrict__ tclst, const double* __restrict__ noise, uint64_t seed,
    double* __restrict__ loss, double* __restrict__ margin, float* __restrict__ normal_out, float* __restrict__ g_q,
    float* __restrict__ g_target, float* __restrict__ g_comp, float* __restrict__ g_tip, int T_rt) {
  constexpr int NTA = NT > 0 ? NT : CDX_MAX_TIPS;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int T = NT > 0 ? NT : T_rt, D = FK ? chain.n_dofs : 0;
  double tp[NTA][3], tg[NTA * 3], cp[NTA], nr[NTA][3];
  for (int f = 0; f < T; ++f) {
    const int64_t r = e * T + f;
    // ½·s1·n1 + ½·s2·n2 and its norm, in float32 (the reference's tensors are float32)
    float n[3];
    const float a1 = 0.5f * (float)sign1[r], a2 = 0.5f * (float)sign2[r];
    for (int i = 0; i < 3; ++i) n[i] = a1 * n1[3 * r + i] + a2 * n2[3 * r + i];
    const float nn = sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (int i = 0; i < 3; ++i) {
      const float v = n[i] / nn;
      nr[f][i] = (double)v;
      if (normal_out) normal_out[3 * r + i] = v;
      tp[f][i] = (double)tip[3 * r + i];
      tg[3 * f + i] = (double)target[3 * r + i];
    }
    cp[f] = (double)comp[r];
  }
  double nz[9];
  if (noise) {
    for (int i = 0; i < 9; ++i) nz[i] = noise[e * 9 + i];
  } else {
    for (int i = 0; i < 9; ++i) nz[i] = (double)(kin_mix(seed ^ kin_mix((uint64_t)(e * 9 + i))) >> 11) * 0x1.0p-53;
  }
  cdx::ForceEqParams fp;
  fp.cos_mu = (double)p.fe.cos_mu;
  fp.gravity = p.fe.gravity;
  for (int i = 0; i < 3; ++i) fp.com[i] = (double)p.fe.com[i];
  fp.dummy_target_z = (double)p.fe.dummy_target_z;
  fp.dummy_comp = (double)p.fe.dummy_comp;
  cdx::ForceEq<NT> fe;
  fe.forward(fp, T, tp, tg, cp, nr, nz);

  // ---- forward
  double ct[3] = {0, 0, 0}, cg[3] = {0, 0, 0};
  for (int f = 0; f < T; ++f)
    for (int i = 0; i < 3; ++i) { ct[i] += tp[f][i]; cg[i] += tg[3 * f + i]; }
  double cd[3];
  for (int i = 0; i < 3; ++i) cd[i] = ct[i] / T - cg[i] / T;
  const double cn = sqrt(cd[0] * cd[0] + cd[1] * cd[1] + cd[2] * cd[2]);
  double dq2 = 0.0;
  for (int i = 0; i < D; ++i) {
    const double d = (double)q[e * D + i] - (double)p.ref_q[i];
    dq2 += d * d;
  }
  const double qn = sqrt(dq2);
  double dcost = 0.0, tcost = 0.0, sd[NTA], std_[NTA];
  for (int f = 0; f < T; ++f) {
    const int64_t r = e * T + f;
    sd[f] = sqrt((double)sqd[r]);
    std_[f] = sqrt((double)tsqd[r]);
    dcost += sd[f];
    tcost += (double)tsign[r] * std_[f];
  }
  const double* fn = fe.fn;
  double zmax = -fn[0];
  for (int f = 1; f < T; ++f) zmax = -fn[f] > zmax ? -fn[f] : zmax;
  double ez[NTA], esum = 0.0;
  for (int f = 0; f < T; ++f) { ez[f] = exp(-fn[f] - zmax); esum += ez[f]; }
  double sm[NTA], v[NTA], fcost = 0.0;
  for (int f = 0; f < T; ++f) {
    sm[f] = ez[f] / esum;
    v[f] = fn[f] * sm[f];
    fcost += v[f] > 1.0 ? 1.0 : v[f];
  }
  // Kin mode adds the joint-space ref_cost last (:205); SDF mode (no chain) has none (:218)
  loss[e] = FK ? -fe.reward * 5.0 + 1000.0 * dcost + 10.0 * tcost + cn * 10.0 - fcost + qn * 10.0
               : -fe.reward * 5.0 + 1000.0 * dcost + 10.0 * tcost + cn * 10.0 - fcost;
  for (int f = 0; f < T; ++f) margin[e * T + f] = fe.margin[f];

  // ---- backward (dl = 1)
  double gt[NTA][3], gg[NTA][3], gc[NTA];
  for (int f = 0; f < T; ++f) {
    const int64_t r = e * T + f;
    gc[f] = 0.0;
    const double gd = 1000.0 * 0.5 / sd[f], gtd = 10.0 * (double)tsign[r] * 0.5 / std_[f];
    for (int i = 0; i < 3; ++i) {
      const double gcen = cn > 0 ? 10.0 * cd[i] / cn / T : 0.0;
      gt[f][i] = 2.0 * gd * (tp[f][i] - (double)clst[3 * r + i]) + gcen;
      gg[f][i] = 2.0 * gtd * (tg[3 * f + i] - (double)tclst[3 * r + i]) - gcen;
    }
  }
  double g_fn[NTA], g_sm[NTA], gsm_dot = 0.0;
  for (int f = 0; f < T; ++f) {
    const double gv = v[f] <= 1.0 ? -1.0 : 0.0;
    g_fn[f] = gv * sm[f];
    g_sm[f] = gv * fn[f];
    gsm_dot += g_sm[f] * sm[f];
  }
  for (int f = 0; f < T; ++f) g_fn[f] += -(sm[f] * (g_sm[f] - gsm_dot));
  fe.backward(-5.0, g_fn, cp, gt, gg, gc);
  if constexpr (FK) {
    float gq[CDX_MAX_DOFS];
    for (int i = 0; i < D; ++i) {
      const double d = (double)q[e * D + i] - (double)p.ref_q[i];
      gq[i] = qn > 0 ? (float)(10.0 * d / qn) : 0.f;
    }
    float fk_g[CDX_MAX_DOFS];
    for (int i = 0; i < D; ++i) fk_g[i] = 0.f;
    for (int f = 0; f < T; ++f) {
      const float gpos[3] = {(float)gt[f][0], (float)gt[f][1], (float)gt[f][2]};
      cdx::fk_tip_bwd<MAXD>(chain, f, q + e * D, gpos, cdx::GqAdd{fk_g});
    }
    for (int i = 0; i < D; ++i) g_q[e * D + i] = gq[i] + fk_g[i];
  }
  if (g_tip)
    for (int f = 0; f < T; ++f)
      for (int i = 0; i < 3; ++i) g_tip[(e * T + f) * 3 + i] = (float)gt[f][i];
  for (int f = 0; f < T; ++f) {
    g_comp[e * T + f] = (float)gc[f];
    for (int i = 0; i < 3; ++i) g_target[(e * T + f) * 3 + i] = (float)gg[f][i];
  }
}


// Four-fingertip variant: four lanes per candidate (lane f = fingertip f), so E = 16 384 candidates fill 1 024
// waves instead of 256.  Every lane of a candidate gathers the candidate's four rows (shuffles) and runs the
// force-equilibrium reward and the cost terms forward and backward itself — identical inputs, identical
// results, no divergence (the lanes would idle otherwise) — then takes its own fingertip's gradients and walks
// its own FK chain backward; the four chains' joint gradients are summed across the lanes ((f0 + f1) + (f2 + f3)).
//
// STEP (cdx_kin_iteration: Kin mode — FK, Adam, no box clamp — or SDF mode — no FK, RMSprop, box clamps): the
// iteration's cdx_kin_step in the same launch — the
// candidate's four lanes hold its loss and every gradient when the cost is done, so the best-iterate update, the
// Adam step of the DOFs / targets / compliances each lane owns and the next fingertip's FK follow without a second
// launch or a gradient round trip through memory.  Same operations in the same order as the two launches:
// bit-identical parameters, best iterate and fingertips.  (q / tip / target / comp alias sb's pose / tips / target /
// comp: a lane reads its candidate's rows before any of the candidate's lanes rewrites them.)
template <int MAXD, bool FK, bool STEP = false>
__global__ __launch_bounds__(64) void kin_cost4_kernel(
    cdx_chain chain, cdx_kin_params p, int64_t E, const float* q, const float* tip, const float* target,
    const float* comp, const int32_t* __restrict__ sign1,
    const float* __restrict__ n1, const float* __restrict__ sqd, const int32_t* __restrict__ sign2,
    const float* __restrict__ n2, const float* __restrict__ clst, const float* __restrict__ tsqd,
    const int32_t* __restrict__ tsign, const float* __restrict__ tclst, const double* __restrict__ noise, uint64_t seed,
    double* __restrict__ loss, double* __restrict__ margin, float* __restrict__ normal_out, float* __restrict__ g_q,
    float* __restrict__ g_target, float* __restrict__ g_comp, float* __restrict__ g_tip, cdx_kin_opt cfg,
    cdx_kin_opt_buffers sb, int it) {
  constexpr int NT = 4;
  if constexpr (STEP && FK) KIN_PHASE(0);
#if !defined(CDX_KIN_FK_BWD1)
  __shared__ float s_fk[CDX_MAX_DOFS][64];  // per-DOF FK gradient contributions (then, with STEP, the summed ones)
#endif
#if !defined(CDX_KIN_FK_BWD1) && !defined(CDX_KIN_FK_BWD2)
  // the FK walk's slots (fk_tip_walk3s) behind the final pose; with STEP, the whole FK-walk cache image (FKS_BLOCK)
  __shared__ float s_jst[fks_slots(MAXD) * 64];
#endif
  __shared__ float s_qn[64 / NT][CDX_MAX_DOFS];  // STEP: the candidates' joint rows (cache check), then the updated rows
  // STEP: the step's operands, prefetched (DOFs f + 4u of the candidate's row, this lane's target / compliance)
  constexpr int PF_DOFS = CDX_MAX_DOFS / NT;
  float pf_p[PF_DOFS], pf_m[PF_DOFS], pf_v[PF_DOFS], pf_t[3], pf_tm[3], pf_tv[3], pf_c = 0.f, pf_cm = 0.f, pf_cv = 0.f;
  float pf_ov = 0.f, pf_nm[3] = {0.f, 0.f, 0.f};
  double pf_mg = 0.0;
  unsigned pf_any = 0u;
  const int64_t tg_ = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e_raw = tg_ >> 2;
  const int f = (int)(tg_ & 3);
  const bool on = e_raw < E;
  const int64_t e = on ? e_raw : E - 1;  // (lanes past E shadow the last candidate: every lane shuffles)
  const int base = (int)(threadIdx.x & ~3u);
  const int D = FK ? chain.n_dofs : 0;
  const int64_t r = e * NT + f;
  // this lane's fingertip row: ½·s1·n1 + ½·s2·n2 and its norm in float32 (the reference's tensors are float32)
  double nro[3], tpo[3], tgo[3];
  {
    float n[3];
    const float a1 = 0.5f * (float)sign1[r], a2 = 0.5f * (float)sign2[r];
    for (int i = 0; i < 3; ++i) n[i] = a1 * n1[3 * r + i] + a2 * n2[3 * r + i];
    const float nn = sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (int i = 0; i < 3; ++i) {
      const float v = n[i] / nn;
      nro[i] = (double)v;
      if (normal_out && on) normal_out[3 * r + i] = v;
      tpo[i] = (double)tip[3 * r + i];
      tgo[i] = (double)target[3 * r + i];
    }
  }
  const double cpo = (double)comp[r], sdo = sqrt((double)sqd[r]), stdo = sqrt((double)tsqd[r]);
  const double tso = (double)tsign[r];
  double tp[NT][3], tg[NT * 3], cp[NT], nr[NT][3], sd[NT], std_[NT], ts[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    const int l = base + k;
    for (int i = 0; i < 3; ++i) {
      tp[k][i] = __shfl(tpo[i], l);
      tg[3 * k + i] = __shfl(tgo[i], l);
      nr[k][i] = __shfl(nro[i], l);
    }
    cp[k] = __shfl(cpo, l);
    sd[k] = __shfl(sdo, l);
    std_[k] = __shfl(stdo, l);
    ts[k] = __shfl(tso, l);
  }
  double nz[9];
  if (noise) {
    for (int i = 0; i < 9; ++i) nz[i] = noise[e * 9 + i];
  } else {
    for (int i = 0; i < 9; ++i) nz[i] = (double)(kin_mix(seed ^ kin_mix((uint64_t)(e * 9 + i))) >> 11) * 0x1.0p-53;
  }
#if !defined(CDX_KIN_FK_BWD1) && !defined(CDX_KIN_FK_BWD2)
  // STEP (Kin): the previous iteration's FK-walk cache of this workgroup and the candidates' current joint rows, into
  // LDS by DMA now — they land while the reward runs; the FK backward checks them and skips the chain walk
  const bool fks = STEP && FK && it > 0 && sb.fk_state != nullptr;
  unsigned fks_tg = 0u;
  if (fks) {
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const float* gb = sb.fk_state + (int64_t)blockIdx.x * FKS_BLOCK;
    fks_tg = reinterpret_cast<const unsigned*>(gb)[fks_at(fks_tag(MAXD), threadIdx.x)];
#pragma unroll
    for (int c = 0; c < fks_slots(MAXD) / 4; ++c)
      __builtin_amdgcn_global_load_lds(gb + 256 * c + 4 * threadIdx.x, (lds_ptr)(s_jst + 256 * c), 16, 0, 0);
    // rows e0 … e0 + 15 (16·D floats, contiguous from pose + e0·D; 16-byte units past the block or past E·D re-read
    // the first unit: those LDS words belong to no live candidate)
    const int64_t e0 = (int64_t)blockIdx.x * (64 / NT);
    const float* qb = sb.pose + e0 * D;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int64_t u = 64 * c + threadIdx.x;
      const bool in = 4 * u + 4 <= (int64_t)(64 / NT) * D && (e0 * D + 4 * u + 4) <= E * D;
      __builtin_amdgcn_global_load_lds(qb + (in ? 4 * u : 0), (lds_ptr)(&s_qn[0][0] + 256 * c), 16, 0, 0);
    }
  }
#endif
  if constexpr (STEP && FK) KIN_PHASE(1);
  cdx::ForceEqParams fp;
  fp.cos_mu = (double)p.fe.cos_mu;
  fp.gravity = p.fe.gravity;
  for (int i = 0; i < 3; ++i) fp.com[i] = (double)p.fe.com[i];
  fp.dummy_target_z = (double)p.fe.dummy_target_z;
  fp.dummy_comp = (double)p.fe.dummy_comp;
  cdx::ForceEq<NT, -1, FeReal> fe;
#if defined(CDX_KIN_FE_F32)
  FeReal cpf[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) cpf[k] = (FeReal)cp[k];
  {
    FeReal tpf[NT][3], tgf[NT * 3], nrf[NT][3];  // (the reference's float32 values: exact)
#pragma unroll
    for (int k = 0; k < NT; ++k)
      for (int i = 0; i < 3; ++i) { tpf[k][i] = (FeReal)tp[k][i]; tgf[3 * k + i] = (FeReal)tg[3 * k + i]; nrf[k][i] = (FeReal)nr[k][i]; }
    fe.forward(fp, NT, tpf, tgf, cpf, nrf, nz);
  }
#elif !defined(CDX_KIN_DIAG_NOFE)
  fe.forward(fp, NT, tp, tg, cp, nr, nz);
#endif
  if constexpr (STEP && FK) KIN_PHASE(2);

  // ---- forward
  double ct[3] = {0, 0, 0}, cg[3] = {0, 0, 0};
  for (int k = 0; k < NT; ++k)
    for (int i = 0; i < 3; ++i) { ct[i] += tp[k][i]; cg[i] += tg[3 * k + i]; }
  double cd[3];
  for (int i = 0; i < 3; ++i) cd[i] = ct[i] / NT - cg[i] / NT;
  const double cn = sqrt(cd[0] * cd[0] + cd[1] * cd[1] + cd[2] * cd[2]);
  double dq2 = 0.0;
  for (int i = 0; i < D; ++i) {
    const double d = (double)q[e * D + i] - (double)p.ref_q[i];
    dq2 += d * d;
  }
  const double qn = sqrt(dq2);
  double dcost = 0.0, tcost = 0.0;
  for (int k = 0; k < NT; ++k) {
    dcost += sd[k];
    tcost += ts[k] * std_[k];
  }
#if defined(CDX_KIN_FE_F32)
  double fn[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) fn[k] = (double)fe.fn[k];
#else
  const double* fn = fe.fn;
#endif
  double zmax = -fn[0];
  for (int k = 1; k < NT; ++k) zmax = -fn[k] > zmax ? -fn[k] : zmax;
  double ez[NT], esum = 0.0;
  for (int k = 0; k < NT; ++k) { ez[k] = exp(-fn[k] - zmax); esum += ez[k]; }
  double sm[NT], v[NT], fcost = 0.0;
  for (int k = 0; k < NT; ++k) {
    sm[k] = ez[k] / esum;
    v[k] = fn[k] * sm[k];
    fcost += v[k] > 1.0 ? 1.0 : v[k];
  }
  const double rw = (double)fe.reward;
  const double lval = FK ? -rw * 5.0 + 1000.0 * dcost + 10.0 * tcost + cn * 10.0 - fcost + qn * 10.0
                         : -rw * 5.0 + 1000.0 * dcost + 10.0 * tcost + cn * 10.0 - fcost;
  if (on && f == 0) loss[e] = lval;
  double mo = 0.0;
  for (int k = 0; k < NT; ++k) mo = k == f ? (double)fe.margin[k] : mo;
  if (on) margin[r] = mo;

  if constexpr (STEP && FK) KIN_PHASE(3);
  // ---- backward (dl = 1)
  double gt[NT][3], gg[NT][3], gc[NT];
  for (int k = 0; k < NT; ++k) {
    const int64_t rk = e * NT + k;
    gc[k] = 0.0;
    const double gd = 1000.0 * 0.5 / sd[k], gtd = 10.0 * ts[k] * 0.5 / std_[k];
    for (int i = 0; i < 3; ++i) {
      const double gcen = cn > 0 ? 10.0 * cd[i] / cn / NT : 0.0;
      gt[k][i] = 2.0 * gd * (tp[k][i] - (double)clst[3 * rk + i]) + gcen;
      gg[k][i] = 2.0 * gtd * (tg[3 * k + i] - (double)tclst[3 * rk + i]) - gcen;
    }
  }
  double g_fn[NT], g_sm[NT], gsm_dot = 0.0;
  for (int k = 0; k < NT; ++k) {
    const double gv = v[k] <= 1.0 ? -1.0 : 0.0;
    g_fn[k] = gv * sm[k];
    g_sm[k] = gv * fn[k];
    gsm_dot += g_sm[k] * sm[k];
  }
  for (int k = 0; k < NT; ++k) g_fn[k] += -(sm[k] * (g_sm[k] - gsm_dot));
#if defined(CDX_KIN_FE_F32)
  {
    FeReal g_fnf[NT], gtf[NT][3], ggf[NT][3], gcf[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      g_fnf[k] = (FeReal)g_fn[k];
      gcf[k] = FeReal(0);
      for (int i = 0; i < 3; ++i) gtf[k][i] = ggf[k][i] = FeReal(0);
    }
    fe.backward(FeReal(-5.0), g_fnf, cpf, gtf, ggf, gcf);
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      for (int i = 0; i < 3; ++i) { gt[k][i] += (double)gtf[k][i]; gg[k][i] += (double)ggf[k][i]; }
      gc[k] += (double)gcf[k];
    }
  }
#elif !defined(CDX_KIN_DIAG_NOFE)
  fe.backward(-5.0, g_fn, cp, gt, gg, gc);
#endif
  if constexpr (STEP && FK) KIN_PHASE(4);
  // this lane's fingertip (selects: no dynamic register indexing)
  double gto[3] = {0, 0, 0}, ggo[3] = {0, 0, 0}, gco = 0.0;
#pragma unroll
  for (int k = 0; k < NT; ++k)
    if (k == f) {
      for (int i = 0; i < 3; ++i) { gto[i] = gt[k][i]; ggo[i] = gg[k][i]; }
      gco = gc[k];
    }
  if constexpr (FK) {
#if defined(CDX_KIN_FK_BWD1)  // (A/B: the stored-rotations backward walk, per-DOF sums in a register array)
    float fk_g[CDX_MAX_DOFS];
    for (int i = 0; i < D; ++i) fk_g[i] = 0.f;
    const float gpos[3] = {(float)gto[0], (float)gto[1], (float)gto[2]};
#if !defined(CDX_KIN_DIAG_NOFK)  // (timing-only diagnostic builds: outputs wrong)
    cdx::fk_tip_bwd<MAXD>(chain, f, q + e * D, gpos, cdx::GqAdd{fk_g});
#endif
#else  // the closed-form backward (fk_tip_bwd2), per-DOF sums in LDS (a register array indexed by DOF spilled)
    for (int i = 0; i < D; ++i) s_fk[i][threadIdx.x] = 0.f;
    const float gpos[3] = {(float)gto[0], (float)gto[1], (float)gto[2]};
#if !defined(CDX_KIN_DIAG_NOFK)
    // the chain read in place from the kernel-argument segment (it is the first argument, at offset 0): indexed by a
    // per-lane body index, the by-value copy went to scratch (≈ 2 KB per lane) in the deep-chain instantiation
    const cdx_chain& kc = *(const cdx_chain*)(__builtin_amdgcn_kernarg_segment_ptr());
    if constexpr (STEP) {
      // the step's operands, loaded now so that their latency hides under the FK backward (the kernel runs at one
      // wave per SIMD): none of them is written before the step reads it
      pf_any = it > 0 ? sb.any[(it - 1) % 3] : 0u;
      pf_ov = sb.opt_value[e];
#pragma unroll
      for (int u = 0; u < PF_DOFS; ++u) {
        const int i = f + NT * u;
        const int64_t k = e * D + (i < D ? i : 0);  // (padded slots re-read DOF 0 of the row)
        pf_p[u] = sb.pose[k];
        pf_m[u] = sb.m_pose[k];
        pf_v[u] = sb.v_pose[k];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pf_t[i] = sb.target[3 * r + i];
        pf_tm[i] = sb.m_target[3 * r + i];
        pf_tv[i] = sb.v_target[3 * r + i];
      }
      pf_c = sb.comp[r];
      pf_cm = sb.m_comp[r];
      pf_cv = sb.v_comp[r];
      if constexpr (FK)
        if (it > 0) {  // the previous iteration's margin / normal slot, which the step commits when any improved
          const bool ps = ((it - 1) & 1) != 0;
          pf_mg = (ps ? sb.margin[1] : sb.margin[0])[r];
          const float* nm = ps ? sb.normal[1] : sb.normal[0];
          for (int i = 0; i < 3; ++i) pf_nm[i] = nm[3 * r + i];
        }
    }
#if defined(CDX_KIN_FK_BWD2)  // (A/B: two walks, no per-level state)
    cdx::fk_tip_bwd2<MAXD>(kc, f, q + e * D, gpos, [&](int d, float v) { s_fk[d][threadIdx.x] += v; });
#else  // one walk, each joint's world axis and origin kept in LDS
    auto gacc = [&](int d, float v) { s_fk[d][threadIdx.x] += v; };
    // the joints' slots in s_jst, in the cache's layout (fks_at)
    auto jput = [&](int l, int i, float v) { s_jst[fks_at(12 + 6 * l + i, threadIdx.x)] = v; };
    auto jget = [&](int l, int i) { return s_jst[fks_at(12 + 6 * l + i, threadIdx.x)]; };
    bool cached = false;
    if constexpr (STEP && FK) KIN_PHASE(12);
    if (fks) {
      // the cache holds this candidate's walk if the previous iteration wrote it (the tag) and the joint row it was
      // walked on has the current row's bits (every lane checks its DOFs f + 4u, the candidate's four lanes agree); a
      // row rewritten since (another entry point's step, a caller) fails the check and walks
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const float* qc = &s_qn[0][0] + (threadIdx.x / NT) * D;
      int okl = fks_tg == (unsigned)it;
#pragma unroll
      for (int u = 0; u < FKS_PF; ++u) {
        const int i = f + NT * u;
        if (i < D && __float_as_uint(s_jst[fks_at(12 + 6 * MAXD + u, threadIdx.x)]) != __float_as_uint(qc[i])) okl = 0;
      }
      okl &= __shfl_xor(okl, 1);
      okl &= __shfl_xor(okl, 2);
      cached = okl != 0;
    }
    if constexpr (STEP && FK) KIN_PHASE(13);
    if (cached) {
      float R[9], t[3];
      for (int i = 0; i < 9; ++i) R[i] = s_jst[fks_at(i, threadIdx.x)];
      for (int i = 0; i < 3; ++i) t[i] = s_jst[fks_at(9 + i, threadIdx.x)];
      cdx::fk_tip_bwd3_grad(kc, f, R, t, gpos, gacc, jget);
    } else {
      float R[9], t[3];
      cdx::fk_tip_walk3s(kc, f, q + e * D, R, t, jput);
      cdx::fk_tip_bwd3_grad(kc, f, R, t, gpos, gacc, jget);
    }
#endif
#endif
    if constexpr (STEP && FK) KIN_PHASE(14);
    float* fk_g = nullptr;
    (void)fk_g;
#endif
#if !defined(CDX_KIN_FK_BWD1)
    if constexpr (STEP) {
      // the same sums, DOF by DOF; a lane's own DOFs f + 4u take their joint angle from the step's prefetch (the
      // loop below re-reads q per DOF behind the previous DOF's g_q store, which q may alias: one load latency each)
#pragma unroll
      for (int u = 0; u < PF_DOFS; ++u)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int i = NT * u + j;
          if (i >= D) break;
          float s = s_fk[i][threadIdx.x];
          s += __shfl_xor(s, 1);
          s += __shfl_xor(s, 2);
          if (j == f) {
            const double d = (double)pf_p[u] - (double)p.ref_q[i];
            const float gq = qn > 0 ? (float)(10.0 * d / qn) : 0.f;
            if (on) g_q[e * D + i] = gq + s;
            s_fk[i][threadIdx.x] = gq + s;  // (this lane's own slot: the step below reads it)
          }
        }
    } else
#endif
    for (int i = 0; i < D; ++i) {
#if defined(CDX_KIN_FK_BWD1)
      float s = fk_g[i];
#else
      float s = s_fk[i][threadIdx.x];
#endif
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      if ((i & 3) == f) {
        const double d = (double)q[e * D + i] - (double)p.ref_q[i];
        const float gq = qn > 0 ? (float)(10.0 * d / qn) : 0.f;
        if (on) g_q[e * D + i] = gq + s;
#if !defined(CDX_KIN_FK_BWD1)
        if constexpr (STEP) s_fk[i][threadIdx.x] = gq + s;  // (this lane's own slot: the step below reads it)
#endif
      }
    }
  }
  if constexpr (STEP && FK) KIN_PHASE(5);
  if (on) {
    if (g_tip)
      for (int i = 0; i < 3; ++i) g_tip[3 * r + i] = (float)gto[i];
    g_comp[r] = (float)gco;
    for (int i = 0; i < 3; ++i) g_target[3 * r + i] = (float)ggo[i];
  }
#if !defined(CDX_KIN_FK_BWD1)
  if constexpr (STEP && FK) {
    // ---- cdx_kin_step's iteration `it` (kin_step_kernel, rule 0, T = 4): the previous iteration's margin / normal
    // commit, the best iterate, Adam, the next fingertip
    if (pf_any && on) {  // (prefetched with the step's operands)
      sb.opt_margin[r] = pf_mg;
      for (int i = 0; i < 3; ++i) sb.opt_normal[3 * r + i] = pf_nm[i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) sb.any[(it + 1) % 3] = 0u;
    const bool flag = on && lval < (double)pf_ov;
    if (flag) {
      if (f == 0) sb.opt_value[e] = (float)lval;
#pragma unroll
      for (int u = 0; u < PF_DOFS; ++u)
        if (f + NT * u < D) sb.opt_pose[e * D + f + NT * u] = pf_p[u];
      for (int i = 0; i < 3; ++i) sb.opt_target[3 * r + i] = pf_t[i];
      sb.opt_comp[r] = pf_c;
    }
    if (__any(flag) && threadIdx.x == 0) atomicOr(sb.any + it % 3, 1u);
    const AdamConst ac = adam_const(cfg, it);
    float* qs = s_qn[threadIdx.x / NT];  // the candidates' updated joint rows, for the FK
#pragma unroll
    for (int u = 0; u < PF_DOFS; ++u) {
      const int i = f + NT * u;
      if (i >= D) break;
      float qv = pf_p[u];
      if (cfg.lr[0] != 0.0) {
        float m = pf_m[u], v = pf_v[u];
        qv = adam_f32(qv, s_fk[i][threadIdx.x], m, v, ac.w1, ac.b2, ac.w2, ac.bc2s, ac.eps, ac.sz[0]);
        if (on) {
          sb.m_pose[e * D + i] = m;
          sb.v_pose[e * D + i] = v;
        }
      }
      if (on) sb.pose[e * D + i] = qv;
      qs[i] = qv;
    }
    if (on) {
      if (cfg.lr[1] != 0.0)
        for (int i = 0; i < 3; ++i) {
          float m = pf_tm[i], v = pf_tv[i];
          sb.target[3 * r + i] = adam_f32(pf_t[i], (float)ggo[i], m, v, ac.w1, ac.b2, ac.w2, ac.bc2s, ac.eps, ac.sz[1]);
          sb.m_target[3 * r + i] = m;
          sb.v_target[3 * r + i] = v;
        }
      if (cfg.lr[2] != 0.0) {
        float m = pf_cm, v = pf_cv;
        sb.comp[r] = adam_f32(pf_c, (float)gco, m, v, ac.w1, ac.b2, ac.w2, ac.bc2s, ac.eps, ac.sz[2]);
        sb.m_comp[r] = m;
        sb.v_comp[r] = v;
      }
    }
    KIN_PHASE(6);
    __syncthreads();
    KIN_PHASE(11);
    if (sb.tips) {
      const cdx_chain& kc = *(const cdx_chain*)(__builtin_amdgcn_kernarg_segment_ptr());
      float pos[3];
      if (sb.fk_state) {  // the walk, kept for the next iteration's FK backward (every lane: its own slots)
        // the walk's slots into this lane's image in s_jst (the backward is done with it), then the lane's whole image
        // to memory after the walk — stores inside it would make each level's chain-descriptor load wait for them
        // (one vmcnt) — one dwordx4 per four slots
        float R[9], t[3];
        KIN_PHASE(8);
        cdx::fk_tip_walk3s(kc, f, QRowLds{qs}, R, t,
                           [&](int l, int i, float v) { s_jst[fks_at(12 + 6 * l + i, threadIdx.x)] = v; });
        KIN_PHASE(9);
        cdx::tip_from_pose(kc, f, R, t, pos, nullptr);
        for (int i = 0; i < 9; ++i) s_jst[fks_at(i, threadIdx.x)] = R[i];
        for (int i = 0; i < 3; ++i) s_jst[fks_at(9 + i, threadIdx.x)] = t[i];
#pragma unroll
        for (int u = 0; u < FKS_PF; ++u) s_jst[fks_at(12 + 6 * MAXD + u, threadIdx.x)] = f + NT * u < D ? qs[f + NT * u] : 0.f;
        const float4* l4 = reinterpret_cast<const float4*>(s_jst) + threadIdx.x;
        float4* gb4 = reinterpret_cast<float4*>(sb.fk_state + (int64_t)blockIdx.x * FKS_BLOCK) + threadIdx.x;
#pragma unroll
        for (int c = 0; c < fks_slots(MAXD) / 4; ++c) gb4[64 * c] = l4[64 * c];
        reinterpret_cast<unsigned*>(sb.fk_state + (int64_t)blockIdx.x * FKS_BLOCK)[fks_at(fks_tag(MAXD), threadIdx.x)] =
            (unsigned)it + 1u;
        KIN_PHASE(10);
      } else {
        cdx::fk_tip(kc, f, QRowLds{qs}, pos, nullptr);
      }
      if (on)
        for (int i = 0; i < 3; ++i) sb.tips[3 * r + i] = pos[i] + cfg.palm_offset[i];
    }
    KIN_PHASE(7);
  }
#endif
  if constexpr (STEP && !FK) {
    // ---- cdx_kin_step's iteration `it` for the SDF optimiser (kin_step_kernel, rule 1, T = 4): the previous
    // iteration's margin / normal commit, the best iterate, RMSprop on this lane's fingertip / target / compliance,
    // the box clamps
    const float pv[3] = {sb.pose[3 * r], sb.pose[3 * r + 1], sb.pose[3 * r + 2]};
    const float tv[3] = {sb.target[3 * r], sb.target[3 * r + 1], sb.target[3 * r + 2]};
    const float cv = sb.comp[r];
    if (it > 0 && sb.any[(it - 1) % 3] && on) {
      const bool ps = ((it - 1) & 1) != 0;
      const double* mg = ps ? sb.margin[1] : sb.margin[0];
      const float* nm = ps ? sb.normal[1] : sb.normal[0];
      sb.opt_margin[r] = mg[r];
      for (int i = 0; i < 3; ++i) sb.opt_normal[3 * r + i] = nm[3 * r + i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) sb.any[(it + 1) % 3] = 0u;
    const bool flag = on && lval < (double)sb.opt_value[e];
    if (flag) {
      if (f == 0) sb.opt_value[e] = (float)lval;
      for (int i = 0; i < 3; ++i) {
        sb.opt_pose[3 * r + i] = pv[i];
        sb.opt_target[3 * r + i] = tv[i];
      }
      sb.opt_comp[r] = cv;
    }
    if (__any(flag) && threadIdx.x == 0) atomicOr(sb.any + it % 3, 1u);
    if (on) {
      const float a = (float)cfg.alpha, w2 = (float)(1.0 - cfg.alpha), eps = (float)cfg.eps;
      auto upd = [&](float* pp, float p0, float g, float* vv, int64_t k, int grp) {
        if (cfg.lr[grp] == 0.0) return;
        float v = vv[k];
        pp[k] = rmsprop_f32(p0, g, v, a, w2, eps, (float)(-cfg.lr[grp]));
        vv[k] = v;
      };
      for (int i = 0; i < 3; ++i) upd(sb.pose, pv[i], (float)gto[i], sb.v_pose, 3 * r + i, 0);
      for (int i = 0; i < 3; ++i) upd(sb.target, tv[i], (float)ggo[i], sb.v_target, 3 * r + i, 1);
      upd(sb.comp, cv, (float)gco, sb.v_comp, r, 2);
      if (cfg.clamp_box)  // (:312-314) torch.clamp: NaN stays NaN
        for (int i = 0; i < 3; ++i) {
          const float lo = cfg.box_lb[3 * f + i], hi = cfg.box_ub[3 * f + i];
          float x = sb.target[3 * r + i];
          x = x < lo ? lo : x;
          sb.target[3 * r + i] = x > hi ? hi : x;
          float y = sb.pose[3 * r + i];
          y = y < lo ? lo : y;
          sb.pose[3 * r + i] = y > hi ? hi : y;
        }
    }
  }
}

}  // namespace

extern "C" int cdx_kin_cost(const cdx_chain* chain, const cdx_kin_params* p, int64_t E, const float* q, const float* tip,
                            const float* target, const float* comp, const int32_t* sign1, const float* n1,
                            const float* sqdist, const int32_t* sign2, const float* n2, const float* clst,
                            const float* tsqdist, const int32_t* tsign, const float* tclst, const double* noise,
                            uint64_t seed, double* loss, double* margin, float* normal, float* g_q, float* g_target,
                            float* g_comp, float* g_tip, cdx_stream_t stream) {
  if (!p || p->fe.n_tips < 1 || p->fe.n_tips > CDX_MAX_TIPS) return CDX_EINVAL;
  if (chain && (chain->n_tips != p->fe.n_tips || chain->n_dofs < 0 || chain->n_dofs > CDX_MAX_DOFS ||
                chain->n_bodies < 1 || chain->n_bodies > CDX_MAX_BODIES))
    return CDX_EINVAL;
  if (E < 0) return CDX_EINVAL;
  if (E == 0) return CDX_OK;
  if (!tip || !target || !comp || !sign1 || !n1 || !sqdist || !sign2 || !n2 || !clst || !tsqdist || !tsign || !tclst ||
      !loss || !margin || !g_target || !g_comp || (chain && (!q || !g_q)) || (!chain && !g_tip))
    return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((E + 63) / 64));
  const int T = p->fe.n_tips;
  const cdx_chain c = chain ? *chain : cdx_chain{};
  const bool shallow = !chain || cdx::chain_max_depth(*chain) <= 8;
#define CDX_KIN_LAUNCH(NT, MAXD, FK)                                                                                  \
  hipLaunchKernelGGL((kin_cost_kernel<NT, MAXD, FK>), grid, dim3(64), 0, s, c, *p, E, q, tip, target, comp, sign1, n1, \
                     sqdist, sign2, n2, clst, tsqdist, tsign, tclst, noise, seed, loss, margin, normal, g_q, g_target,    \
                     g_comp, g_tip, T)
#define CDX_KIN4_LAUNCH(MAXD, FK)                                                                                      \
  hipLaunchKernelGGL((kin_cost4_kernel<MAXD, FK>), dim3((unsigned)((4 * E + 63) / 64)), dim3(64), 0, s, c, *p, E, q, tip, \
                     target, comp, sign1, n1, sqdist, sign2, n2, clst, tsqdist, tsign, tclst, noise, seed, loss, margin,   \
                     normal, g_q, g_target, g_comp, g_tip, cdx_kin_opt{}, cdx_kin_opt_buffers{}, 0)
#if defined(CDX_KIN_1LANE)  // A/B: one lane per candidate for four fingertips too (round 4)
  if (!chain && T == 4) CDX_KIN_LAUNCH(4, 8, false);
  else if (!chain) CDX_KIN_LAUNCH(0, 8, false);
  else if (T == 4 && shallow) CDX_KIN_LAUNCH(4, 8, true);
  else if (T == 4) CDX_KIN_LAUNCH(4, CDX_MAX_DEPTH, true);
#else
  if (!chain && T == 4) CDX_KIN4_LAUNCH(8, false);
  else if (!chain) CDX_KIN_LAUNCH(0, 8, false);
  else if (T == 4 && shallow) CDX_KIN4_LAUNCH(8, true);
  else if (T == 4) CDX_KIN4_LAUNCH(CDX_MAX_DEPTH, true);
#endif
  else if (shallow) CDX_KIN_LAUNCH(0, 8, true);
  else CDX_KIN_LAUNCH(0, CDX_MAX_DEPTH, true);
#undef CDX_KIN_LAUNCH
#undef CDX_KIN4_LAUNCH
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

// ------------------------------------------------------------------ Kin / SDF optimiser step
// One launch per iteration after cdx_kin_cost (optimize_pregrasp.py:212-223 Kin, :299-314 SDF): threads
// (candidate e, tip f), T to a candidate, 64 / T candidates to a 64-thread workgroup.
namespace {


__global__ __launch_bounds__(64) void kin_step_kernel(cdx_chain chain, cdx_kin_opt cfg, cdx_kin_opt_buffers b, int64_t E,
                                                      int T, int D, int s, int finalize) {
  __shared__ float s_q[64 * CDX_MAX_DOFS];  // updated joint rows of the workgroup's candidates (G·D ≤ 64·32)
  const int G = 64 / T;
  const int t = threadIdx.x;
  const int gl = t / T, f = t - gl * T;
  const int64_t e = (int64_t)blockIdx.x * G + gl;
  const bool on = gl < G && e < E;
  const int64_t r = e * T + f;
  // commit the previous iteration's margin / normal if some candidate improved in it (its flags are final:
  // that step kernel has finished)
  if (s > 0 && b.any[(s - 1) % 3] && on) {
    const int ps = (s - 1) & 1;
    b.opt_margin[r] = b.margin[ps][r];
    for (int i = 0; i < 3; ++i) b.opt_normal[3 * r + i] = b.normal[ps][3 * r + i];
  }
  if (finalize) return;
  if (blockIdx.x == 0 && t == 0) b.any[(s + 1) % 3] = 0u;  // (written at s − 2, read at s − 1: free now)
  const bool kin = cfg.rule == 0;
  const int npose = kin ? D : 3;               // pose entries this thread owns: q[i], i ≡ f (mod T) / tip f's xyz
  // best iterate (before the step, with the parameters the loss was computed on)
  bool flag = false;
  if (on) {
    const double l = b.loss[e];
    flag = l < (double)b.opt_value[e];
    if (flag) {
      if (f == 0) b.opt_value[e] = (float)l;
      if (kin) {
        for (int i = f; i < D; i += T) b.opt_pose[e * D + i] = b.pose[e * D + i];
      } else {
        for (int i = 0; i < 3; ++i) b.opt_pose[3 * r + i] = b.pose[3 * r + i];
      }
      for (int i = 0; i < 3; ++i) b.opt_target[3 * r + i] = b.target[3 * r + i];
      b.opt_comp[r] = b.comp[r];
    }
  }
  if (__any(flag) && (t & 63) == 0) atomicOr(b.any + s % 3, 1u);
  if (!on) return;
  const double step = (double)(s + 1);
  float w1 = 0.f, b2 = 0.f, w2 = 0.f, bc2s = 1.f, eps = (float)cfg.eps, sz[3] = {0.f, 0.f, 0.f};
  if (kin) {
    const double bc1 = 1.0 - pow(cfg.beta1, step), bc2 = 1.0 - pow(cfg.beta2, step);
    w1 = (float)(1.0 - cfg.beta1);
    b2 = (float)cfg.beta2;
    w2 = (float)(1.0 - cfg.beta2);
    bc2s = (float)sqrt(bc2);
    for (int g = 0; g < 3; ++g) sz[g] = (float)(-(cfg.lr[g] / bc1));
  } else {
    b2 = (float)cfg.alpha;
    w2 = (float)(1.0 - cfg.alpha);
    for (int g = 0; g < 3; ++g) sz[g] = (float)(-cfg.lr[g]);
  }
  auto upd = [&](float* p, const float* g, float* m, float* v, int64_t k, int grp) {
    if (cfg.lr[grp] == 0.0) return;
    p[k] = kin ? adam_f32(p[k], g[k], m[k], v[k], w1, b2, w2, bc2s, eps, sz[grp])
               : rmsprop_f32(p[k], g[k], v[k], b2, w2, eps, sz[grp]);
  };
  // pose: Kin — the joint angles this thread owns, and the whole updated row into LDS for the FK; SDF — tip f
  if (kin) {  // the DOFs i ≡ f (mod T) of the row, each into LDS for the FK below (loads issued ahead of the updates)
    float* qs = s_q + gl * D;
    constexpr int U = 4;
    for (int i0 = f; i0 < D; i0 += U * T) {
      float pv[U], gv[U], mv[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * T;
        const int64_t k = e * D + (i < D ? i : 0);  // (padded slots re-read DOF 0 of the row)
        pv[u] = b.pose[k];
        gv[u] = b.g_pose[k];
        mv[u] = b.m_pose[k];
        vv[u] = b.v_pose[k];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * T;
        if (i >= D) break;
        const int64_t k = e * D + i;
        float qn = pv[u];
        if (cfg.lr[0] != 0.0) {
          qn = adam_f32(qn, gv[u], mv[u], vv[u], w1, b2, w2, bc2s, eps, sz[0]);
          b.m_pose[k] = mv[u];
          b.v_pose[k] = vv[u];
        }
        b.pose[k] = qn;
        qs[i] = qn;
      }
    }
  } else {
    for (int i = 0; i < 3; ++i) upd(b.pose, b.g_pose, b.m_pose, b.v_pose, 3 * r + i, 0);
  }
  for (int i = 0; i < 3; ++i) upd(b.target, b.g_target, b.m_target, b.v_target, 3 * r + i, 1);
  upd(b.comp, b.g_comp, b.m_comp, b.v_comp, r, 2);
  if (cfg.clamp_box)  // (:312-314) torch.clamp: NaN stays NaN
    for (int i = 0; i < 3; ++i) {
      const float lo = cfg.box_lb[3 * f + i], hi = cfg.box_ub[3 * f + i];
      float x = b.target[3 * r + i];
      x = x < lo ? lo : x;
      b.target[3 * r + i] = x > hi ? hi : x;
      if (!kin) {
        float y = b.pose[3 * r + i];
        y = y < lo ? lo : y;
        b.pose[3 * r + i] = y > hi ? hi : y;
      }
    }
  (void)npose;
  if (!kin || !b.tips) return;
  // the next iteration's fingertip f: FK(q) + palm offset (:148)
  __syncthreads();
  float pos[3];
  cdx::fk_tip(chain, f, QRowLds{s_q + gl * D}, pos, nullptr);
  for (int i = 0; i < 3; ++i) b.tips[3 * r + i] = pos[i] + cfg.palm_offset[i];
}

}  // namespace

extern "C" int cdx_kin_step(const cdx_chain* chain, const cdx_kin_opt* cfg, const cdx_kin_opt_buffers* buf, int64_t E,
                            int32_t n_tips, int32_t iteration, int32_t finalize, cdx_stream_t stream) {
  if (!cfg || !buf || E < 0 || n_tips < 1 || n_tips > CDX_MAX_TIPS || iteration < 0 || (cfg->rule != 0 && cfg->rule != 1))
    return CDX_EINVAL;
  const bool kin = cfg->rule == 0;
  if (kin && (!chain || chain->n_tips != n_tips || chain->n_dofs < 1 || chain->n_dofs > CDX_MAX_DOFS ||
              chain->n_bodies < 1 || chain->n_bodies > CDX_MAX_BODIES))
    return CDX_EINVAL;
  if (E == 0) return CDX_OK;
  const cdx_kin_opt_buffers& b = *buf;
  if (!b.margin[0] || !b.margin[1] || !b.normal[0] || !b.normal[1] || !b.opt_margin || !b.opt_normal || !b.any)
    return CDX_EINVAL;
  if (!finalize && (!b.pose || !b.target || !b.comp || !b.g_pose || !b.g_target || !b.g_comp || !b.v_pose ||
                    !b.v_target || !b.v_comp || (kin && (!b.m_pose || !b.m_target || !b.m_comp)) || !b.loss ||
                    !b.opt_value || !b.opt_pose || !b.opt_target || !b.opt_comp))
    return CDX_EINVAL;
  const int G = 64 / n_tips;
  const cdx_chain c = chain ? *chain : cdx_chain{};
  hipLaunchKernelGGL(kin_step_kernel, dim3((unsigned)((E + G - 1) / G)), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     c, *cfg, b, E, (int)n_tips, kin ? (int)chain->n_dofs : 0, (int)iteration, (int)finalize);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

// One optimiser iteration: cdx_kin_cost then cdx_kin_step on the parameters / slots in `buf` — in ONE launch
// (kin_cost4_kernel<…, STEP>) for the Kin optimiser's case (chain, four fingertips, Adam, no box clamp) and the SDF
// optimiser's (no chain, four fingertips, RMSprop, box clamps), else the two launches.

extern "C" int cdx_kin_iteration(const cdx_chain* chain, const cdx_kin_params* p, const cdx_kin_opt* cfg,
                                 const cdx_kin_opt_buffers* buf, int64_t E, int32_t n_tips, const int32_t* sign1,
                                 const float* n1, const float* sqdist, const int32_t* sign2, const float* n2,
                                 const float* clst, const float* tsqdist, const int32_t* tsign, const float* tclst,
                                 const double* noise, uint64_t seed, int32_t iteration, cdx_stream_t stream) {
  if (!p || !cfg || !buf || iteration < 0 || (cfg->rule != 0 && cfg->rule != 1) || n_tips != p->fe.n_tips) return CDX_EINVAL;
  const cdx_kin_opt_buffers& b = *buf;
  const bool kin = cfg->rule == 0;
  if (kin && (!chain || !b.tips)) return CDX_EINVAL;
  float* g_pose = const_cast<float*>(b.g_pose);
  float* g_target = const_cast<float*>(b.g_target);
  float* g_comp = const_cast<float*>(b.g_comp);
  double* loss = const_cast<double*>(b.loss);
  double* margin = b.margin[iteration & 1];
  float* normal = b.normal[iteration & 1];
  // one launch: the Kin optimiser (chain, Adam, no box clamp) or the SDF optimiser (no chain, RMSprop), four tips
  const bool fuse = n_tips == 4 && (kin ? !cfg->clamp_box : !chain);
  if (!fuse) {
    int rc = cdx_kin_cost(kin ? chain : nullptr, p, E, kin ? b.pose : nullptr, kin ? b.tips : b.pose, b.target, b.comp,
                          sign1, n1, sqdist, sign2, n2, clst, tsqdist, tsign, tclst, noise, seed, loss, margin, normal,
                          kin ? g_pose : nullptr, g_target, g_comp, kin ? nullptr : g_pose, stream);
    if (rc) return rc;
    return cdx_kin_step(kin ? chain : nullptr, cfg, buf, E, n_tips, iteration, 0, stream);
  }
  // the two calls' argument checks
  if (E < 0 || (kin && (chain->n_tips != 4 || chain->n_dofs < 1 || chain->n_dofs > CDX_MAX_DOFS ||
                        chain->n_bodies < 1 || chain->n_bodies > CDX_MAX_BODIES)))
    return CDX_EINVAL;
  if (E == 0) return CDX_OK;
  if (!b.pose || !b.target || !b.comp || !g_pose || !g_target || !g_comp || (kin && (!b.m_pose || !b.m_target)) ||
      !b.v_pose ||
      !b.v_target || (kin && !b.m_comp) || !b.v_comp || !loss || !margin || !normal || !b.margin[0] || !b.margin[1] ||
      !b.normal[0] || !b.normal[1] || !b.opt_value || !b.opt_margin || !b.opt_normal || !b.opt_pose || !b.opt_target ||
      !b.opt_comp || !b.any || !sign1 || !n1 || !sqdist || !sign2 || !n2 || !clst || !tsqdist || !tsign || !tclst)
    return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((4 * E + 63) / 64));
#define CDX_KIN4_STEP_LAUNCH(MAXD)                                                                                    \
  hipLaunchKernelGGL((kin_cost4_kernel<MAXD, true, true>), grid, dim3(64), 0, s, *chain, *p, E, b.pose, b.tips,        \
                     b.target, b.comp, sign1, n1, sqdist, sign2, n2, clst, tsqdist, tsign, tclst, noise, seed, loss,     \
                     margin, normal, g_pose, g_target, g_comp, nullptr, *cfg, b, (int)iteration)
  if (!kin)
    hipLaunchKernelGGL((kin_cost4_kernel<8, false, true>), grid, dim3(64), 0, s, cdx_chain{}, *p, E, nullptr, b.pose,
                       b.target, b.comp, sign1, n1, sqdist, sign2, n2, clst, tsqdist, tsign, tclst, noise, seed, loss,
                       margin, normal, nullptr, g_target, g_comp, g_pose, *cfg, b, (int)iteration);
  else if (cdx::chain_max_depth(*chain) <= 8) CDX_KIN4_STEP_LAUNCH(8);
  else CDX_KIN4_STEP_LAUNCH(CDX_MAX_DEPTH);
#undef CDX_KIN4_STEP_LAUNCH
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

extern "C" int64_t cdx_kin_fk_state_bytes(int64_t E, int32_t n_tips) {
  if (E <= 0 || n_tips != 4) return 0;  // (only the four-fingertip one-launch iteration keeps the cache)
  return ((4 * E + 63) / 64) * (int64_t)FKS_BLOCK * (int64_t)sizeof(float);
}

#if defined(CDX_KIN_DIAG_PHASES)
extern "C" int cdx_kin_phase_read(unsigned long long* out) {  // [4096][8] stamps of the last fused Kin iteration
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kin_phase), sizeof(g_kin_phase)) == hipSuccess ? 0 : 1;  // [4096][16]
}
#endif
