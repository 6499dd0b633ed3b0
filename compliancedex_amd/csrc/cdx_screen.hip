// Split-precision screen of the GPIS posterior variance on the bf16 matrix cores (gfx950).
//
// The closure's variance cost reads only max_f log(100·std_f) over a candidate's fingertips
// (optimize_pregrasp.py:733): one fingertip per (level, candidate) reaches the loss and its
// gradient.  The screen estimates std² = k0 − ‖L⁻¹k‖² (gpis.py:56-59, whitened form) for every
// all-tip query at a fraction of the fp64 cost, so that the exact fp64 whitened pass only runs
// for the fingertips that can still be the maximum (cdx_closure, cdx_screen_select below):
//
//   Ṽ = Ã·L⁻ᵀ + k0·colsum(L⁻ᵀ),  Ã = K* − k0   (the offset keeps |Ã| small near the query, where
//                                              the cancellation in k0 − ‖V‖² is worst)
//   Ã and L⁻ᵀ are each split into three bf16 slices (x = x0 + x1 + x2, ≈ 24 bits: Ã exactly, it
//   is generated in fp32), and the six slice products of index sum ≤ 2 are accumulated into one
//   fp32 accumulator per output by v_mfma_f32_32x32x16_bf16 — fp32-level accuracy at 6 bf16
//   MFMAs (2.5 PF/s dense) instead of one fp64 MFMA (78.6 TF/s): 2.1× the flop rate and no f64
//   VALU work on the DP pipe.  Σ Ṽ² is summed in f64.
//
// The estimate carries no parity claim by itself: the closure only uses it to discard fingertips
// whose estimated std² is below the leader's by more than twice the per-object error bound
// (cdx_gpis.screen_delta, calibrated against the fp64 pass when the state is built), and writes
// exact fp64 values for every fingertip it keeps.  tools/screen_emul.py emulates this arithmetic
// bit-for-bit on the CPU (max |Δstd²|/k0 = 1.8e-6 on the config-2 workload).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "cdx_gpis.h"
#include "cdx_gpis_launch.h"
#include "cdx_prof.h"
#include "cdx_screen.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

using cdx::SC_BK;
using cdx::SC_BN;
constexpr int SC_BM = 256;                 // query rows per workgroup
constexpr int SC_THREADS = 512;            // 8 waves: 2 (rows) × 4 (columns), 128 × 64 outputs each
constexpr int SC_REG = 6 * 256;            // 16-byte LDS units of one operand stage: [slice][khalf][256]
constexpr int SC_LDT = 264;               // fp32 row pitch of the epilogue's accumulator image (4 rows ≡ 32 banks)
// LDS: A stages (generated, 2 buffers) | B stages (LDS-DMA ring of 3)
constexpr int SC_A_OFF = 0, SC_B_OFF = 2 * SC_REG * 16;
constexpr int SC_SMEM = std::max(SC_B_OFF + 3 * SC_REG * 16,  // stage buffers
                                 128 * SC_LDT * 4);            // epilogue: one row half of the tile
static_assert(SC_SMEM <= 160 * 1024, "screen stage buffers exceed the CU's LDS");

// K-steps (16 rows of L⁻ᵀ) of stripe nt: rows [0, min(N, (nt+1)·256 − shift)) as in the fp64 pass.
__device__ __host__ inline int sc_ksteps(int nt, int N, int Np) {
  const int hi = std::min(N, (nt + 1) * SC_BN - cdx::screen_shift(N, Np));
  return (hi + SC_BK - 1) / SC_BK;
}

// Ã = k(r) − k(0) in fp32 from a centred fp32 offset (d = x − x_n).
template <int KT>
__device__ __forceinline__ float k_offset(float dx, float dy, float dz, float R, float inv_s2) {
  const float r2 = dx * dx + dy * dy + dz * dz;
  if (KT == CDX_KERNEL_RBF) return expm1f(-0.5f * r2 * inv_s2);
  const float r = __builtin_amdgcn_sqrtf(r2);  // v_sqrt_f32 (≤ 1 ulp): ample for a screen
  const float tps = r2 * (2.0f * r - 3.0f * R);  // 2r³ − 3Rr²  (= TPS − R³)
  if (KT == CDX_KERNEL_TPS) return tps;
  return 0.3f * expm1f(-0.5f * r2 * inv_s2) + 0.7f * tps;
}

// x = s0 + s1 + s2 exactly, each a bf16 given as the high half of an fp32 bit pattern: truncated
// 8-bit pieces of x's 24-bit significand (the remainders are exact in fp32).
__device__ __forceinline__ void split3(float x, unsigned& s0, unsigned& s1, unsigned& s2) {
  s0 = __float_as_uint(x) & 0xffff0000u;
  const float r1 = x - __uint_as_float(s0);
  s1 = __float_as_uint(r1) & 0xffff0000u;
  s2 = __float_as_uint(r1 - __uint_as_float(s1));  // ≤ 8 significant bits: low half already zero
}

// One workgroup per (query tile of 256 rows, stripe of 256 columns); stripes paired heavy+light per
// XCD as in gpis_std_kernel<VAR>.  partial[nt][m] = Σ over the stripe's columns of (Ã·L⁻ᵀ + c)².
template <int KT>
__global__ __launch_bounds__(SC_THREADS, 2) void gpis_screen_kernel(cdx_gpis g, const double* __restrict__ X, int64_t M,
                                                                    double* __restrict__ partial, int64_t M_pad, int Mt,
                                                                    int Nt) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[SC_SMEM];
  u32x4* const sA4 = reinterpret_cast<u32x4*>(smem + SC_A_OFF);  // A buffer b at sA4 + b·SC_REG
  u32x4* const sB4 = reinterpret_cast<u32x4*>(smem + SC_B_OFF);  // B ring slot r at sB4 + r·SC_REG
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Np = g.N_pad, N = g.N;
  const cdx::ScreenView sv = cdx::screen_view(g);
  const int shift = cdx::screen_shift(N, Np);

  // (query tile, stripe): heavy+light stripe pairs per XCD (blocks b, b+8, … share an XCD)
  const int b = blockIdx.x;
  int nt, mt;
  {
    const int Xd = 16 / Nt;
    if (Nt >= 2 && Nt <= 16 && (Nt & (Nt - 1)) == 0 && Mt % Xd == 0) {
      const int xcd = b & 7, r = b >> 3, per = Mt / Xd;
      const int a = xcd / Xd, part = xcd % Xd;
      nt = r < per ? Nt - 1 - a : a;
      mt = part * per + (r < per ? r : r - per);
    } else {
      nt = Nt - 1 - b / Mt;
      mt = b % Mt;
    }
  }
  const int64_t m0 = (int64_t)mt * SC_BM;
  const int n0 = nt * SC_BN;
  const int nK = sc_ksteps(nt, N, Np);

  // generation: thread → query row grow, k-half gkh (wave-uniform), 8 entries per stage
  const int grow = tid & (SC_BM - 1);
  const int gkh = __builtin_amdgcn_readfirstlane(tid >> 8);
  float qx, qy, qz;
  {
    const int64_t m = std::min(m0 + grow, M - 1);  // pad rows replicate a valid query
    qx = (float)(X[3 * m] - sv.center[0]);
    qy = (float)(X[3 * m + 1] - sv.center[1]);
    qz = (float)(X[3 * m + 2] - sv.center[2]);
  }
  const float R = (float)g.R, inv_s2 = (float)(1.0 / (g.sigma * g.sigma));

  // wave → 128 × 64 output sub-tile; waves w and w+4 share a SIMD and take complementary columns
  const int cwave = wave < 4 ? wave : 7 - wave;
  const int wr = (wave >> 2) * 128;
  const int wc = cwave * 64;
  // B rows past this wave's last column are zero (upper-triangular L⁻ᵀ, shifted columns)
  const int kend_w = __builtin_amdgcn_readfirstlane(n0 + wc + 64 - shift);

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Staging by LDS-DMA (global_load_lds: no VGPRs, no ds_write).  issue(st): every wave DMAs 3 × 1 KB
  // of B stage st (instruction u = wave + 8i: slice/k-half region u>>2, columns 64·(u&3) + lane).
  // issue(s+2) runs during step s; the counted `s_waitcnt vmcnt(3)` at the end of each step keeps
  // exactly that step's DMAs in flight across the raw s_barrier (__syncthreads would wait vmcnt(0)),
  // with B stage s+1 landed for step s+1.  Clamped stages past the stripe's end load into free
  // slots, so every step issues the same count.
  const char* Lb = static_cast<const char*>(sv.L);
  auto issue = [&](int st) {
    const int sc = std::min(st, nK - 1);
    const int slot = st % 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int u = wave + 8 * i, reg = u >> 2, col = 64 * (u & 3) + lane;
      const char* src = Lb + (((int64_t)(sc * 6 + reg)) * Np + n0 + col) * 16;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sB4 + slot * SC_REG + u * 64), 16, 0, 0);
    }
  };
  u32x4 ast[3];      // generated A stage: 8 entries × 3 bf16 slices, packed in pairs
  // X1 rows of the generated stage: wave-uniform addresses → scalar loads (SMEM; the vector memory
  // counter stays free for the DMAs' counted waits)
  auto gen_a = [&](int st) {  // 8 consecutive k of this thread's half, packed in pairs
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float4 cfloat4;  // constant space: SMEM loads
#else
    typedef const float4 cfloat4;
#endif
    cfloat4* x1 = (cfloat4*)(sv.X1f) + __builtin_amdgcn_readfirstlane(st * SC_BK + 8 * gkh);
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const float4 p = x1[e], p1 = x1[e + 1];
      unsigned a0, a1, a2, b0, b1, b2;
#if defined(CDX_SC_DIAG_NOGEN)  // timing-only diagnostic build: outputs are wrong
      a0 = __float_as_uint(qx - p.x); a1 = __float_as_uint(qy - p.y); a2 = __float_as_uint(qz - p.z);
      b0 = __float_as_uint(qx - p1.x); b1 = __float_as_uint(qy - p1.y); b2 = __float_as_uint(qz - p1.z);
#else
      split3(k_offset<KT>(qx - p.x, qy - p.y, qz - p.z, R, inv_s2), a0, a1, a2);
      split3(k_offset<KT>(qx - p1.x, qy - p1.y, qz - p1.z, R, inv_s2), b0, b1, b2);
#endif
      ast[0][e / 2] = __builtin_amdgcn_perm(b0, a0, 0x07060302u);
      ast[1][e / 2] = __builtin_amdgcn_perm(b1, a1, 0x07060302u);
      ast[2][e / 2] = __builtin_amdgcn_perm(b2, a2, 0x07060302u);
    }
  };
  auto write_a = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 3; ++i) sA4[buf * SC_REG + (i * 2 + gkh) * 256 + grow] = ast[i];
  };
  // one stage's 48 MFMAs: lane → (row/col l&31, k-half l>>5); B slices of both column blocks, A
  // slice by slice (products of slice-index sum ≤ 2, smallest first)
  auto mfma_stage = [&](int abuf, int bslot, auto more_c) {
    constexpr bool MORE = decltype(more_c)::value;
    bf16x8 fb[3][2];
#pragma unroll
    for (int sb = 0; sb < 3; ++sb)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[sb][j] = __builtin_bit_cast(bf16x8, sB4[bslot * SC_REG + (sb * 2 + (lane >> 5)) * 256 + wc + 32 * j + (lane & 31)]);
#pragma unroll
    for (int sa = 2; sa >= 0; --sa) {
      bf16x8 fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = __builtin_bit_cast(bf16x8, sA4[abuf * SC_REG + (sa * 2 + (lane >> 5)) * 256 + wr + 32 * i + (lane & 31)]);
#pragma unroll
      for (int sb = 2 - sa; sb >= 0; --sb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#if defined(CDX_SC_DIAG_NOMFMA)  // timing-only diagnostic build: outputs are wrong
            acc[i][j][0] += (float)fa[i][0] * (float)fb[sb][j][0];
#else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[sb][j], acc[i][j], 0, 0, 0);
#endif
      if (!MORE) __builtin_amdgcn_sched_barrier(0);  // tail step: no fragment hoisting past a slice group
    }
  };

  // prologue: B stages 0–1 landed, A of stage 0 generated
  issue(0);
  issue(1);
  gen_a(0);
  write_a(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // Step s multiplies stage s (A buffer s&1, B slot s%3) while stage s+2 is DMA'd into slot (s+2)%3
  // and stage s+1's A is generated (X1 slot (s+1)%3) and written to the other A buffer.  LIVE: this
  // wave's B columns are non-zero in stage s; MORE: a stage s+1 exists.  The (LIVE, MORE) body is
  // one straight-line block, so the generation's VALU work interleaves with the MFMAs.
  auto step = [&](int s, auto live_c, auto more_c) {
    constexpr bool LIVE = decltype(live_c)::value, MORE = decltype(more_c)::value;
    issue(s + 2);
    if (MORE) gen_a(s + 1);
    if (LIVE) mfma_stage(s & 1, s % 3, more_c);
    if (MORE) write_a((s + 1) & 1);
    asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");  // B stage s+1 landed, A written
    __builtin_amdgcn_s_barrier();
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const int s_live = std::min(nK, std::max(0, (kend_w + SC_BK - 1) / SC_BK));  // wave-uniform
  int s = 0;
  for (; s < std::min(s_live, nK - 1); ++s) step(s, T_{}, T_{});
  for (; s < nK - 1; ++s) step(s, F_{}, T_{});
  // last stage: its MFMAs only; then every DMA drained before the epilogue reuses the LDS
  if (s < s_live) mfma_stage(s & 1, s % 3, F_{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Epilogue: per row Σ over the stripe's 256 columns of (Ṽ + c)² in f64.  The accumulators go
  // through LDS one row half at a time ([128][SC_LDT] fp32, the stage buffers are free after the
  // loop), then 4 threads per row sum 64 columns each and combine with two xor-shuffles.  (Summing
  // in registers needs the f64 squares of a whole row block live next to the accumulators and
  // made the allocator spill.)  C map (32x32x16): reg r of lane l is row (r&3) + 8(r>>2) + 4(l>>5),
  // column l&31.
  float* T = reinterpret_cast<float*>(smem);
  const int erow = tid >> 2, epart = tid & 3;
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    if (ph) __syncthreads();  // phase 0's readers are done with T
    if ((wave >> 2) == ph) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            T[(32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * SC_LDT + wc + 32 * j + (lane & 31)] = acc[i][j][r];
    }
    __syncthreads();
    const float4* Tr = reinterpret_cast<const float4*>(T + erow * SC_LDT + 64 * epart);
    const double* cs = sv.csum + n0 + 64 * epart;
    double sum = 0.0;
#pragma unroll 4
    for (int c = 0; c < 16; ++c) {
      const float4 v = Tr[c];
      const double x0 = (double)v.x + cs[4 * c], x1 = (double)v.y + cs[4 * c + 1], x2 = (double)v.z + cs[4 * c + 2],
                   x3 = (double)v.w + cs[4 * c + 3];
      sum = fma(x0, x0, sum);
      sum = fma(x1, x1, sum);
      sum = fma(x2, x2, sum);
      sum = fma(x3, x3, sum);
    }
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    if (epart == 0) partial[(int64_t)nt * M_pad + m0 + 128 * ph + erow] = sum;
  }
}

// var[m] = k0 − Σ_nt partial[nt][m] (stripe order).
template <int KT>
__global__ __launch_bounds__(256) void gpis_screen_finalize(cdx_gpis g, const double* __restrict__ partial, int64_t M,
                                                            int64_t M_pad, int Nt, double* __restrict__ var) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  double s = 0;
  for (int t = 0; t < Nt; ++t) s += partial[(int64_t)t * M_pad + m];
  var[m] = cdx::gpis_k0<KT>(g.R) - s;
}

// ------------------------------------------------------------------ closure screening
// Groups of T consecutive all-tip rows (one (distinct level, candidate) each); the variance cost
// takes max_f log(100·std_f) over a group (optimize_pregrasp.py:733).  Per group: s̃²_f = k0 − Σ
// stripe partials; leader = first maximum; the fingertips kept for the exact pass are the leader
// and every f with s̃²_f + Δ ≥ s̃²_lead − Δ (Δ = g.screen_delta ≥ max |s̃² − std²|), or all T when a
// value is not finite or s̃²_lead ≤ 2Δ.  A discarded fingertip gets std = sqrt(max(s̃², 0)), which
// is below the leader's exact std, so the level kernel's own argmax is unchanged.
template <int KT>
__global__ __launch_bounds__(256) void screen_select_kernel(cdx_gpis g, const double* __restrict__ partial,
                                                            int64_t M_pad, int Nt, int64_t G, int T,
                                                            double* __restrict__ sv2, double* __restrict__ std_,
                                                            int* __restrict__ vpos, int* __restrict__ rows,
                                                            unsigned char* __restrict__ keep) {
  const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= G) return;
  const double k0 = cdx::gpis_k0<KT>(g.R), delta = g.screen_delta;
  double s2[CDX_MAX_TIPS];
  bool finite = true;
  int lead = 0;
  for (int f = 0; f < T; ++f) {
    const int64_t q = gi * T + f;
    double acc = 0;
    for (int t = 0; t < Nt; ++t) acc += partial[(int64_t)t * M_pad + q];
    s2[f] = k0 - acc;
    sv2[q] = s2[f];
    finite = finite && isfinite(s2[f]);
    if (s2[f] > s2[lead]) lead = f;
  }
  const bool all = !finite || !(s2[lead] > 2 * delta);
  const double lo = s2[lead] - delta;
  unsigned mask = 0;
  for (int f = 0; f < T; ++f) {
    const int64_t q = gi * T + f;
    if (f == lead) {
      vpos[q] = (int)gi;
      rows[gi] = (int)q;
    } else if (all || s2[f] + delta >= lo) {
      mask |= 1u << f;  // position assigned by screen_compact_kernel
    } else {
      vpos[q] = -1;
      std_[q] = sqrt(fmax(s2[f], 0.0));
    }
  }
  keep[gi] = (unsigned char)mask;
}

// Deterministic compaction of the kept non-leader fingertips behind the G leaders (group order,
// fingertip order): one workgroup scans the per-group counts in chunks of 1024.  stats[0] = their
// number, stats[1] (exact-pass bound violations, refine_select) reset here.
__global__ __launch_bounds__(1024) void screen_compact_kernel(int64_t G, int T, const unsigned char* __restrict__ keep,
                                                              int* __restrict__ vpos, int* __restrict__ rows,
                                                              int* __restrict__ stats) {
  __shared__ int sc[1024];
  const int t = threadIdx.x;
  int carry = 0;
  for (int64_t c0 = 0; c0 < G; c0 += 1024) {
    const int64_t gi = c0 + t;
    const unsigned m = gi < G ? keep[gi] : 0u;
    const int n = __popc(m);
    sc[t] = n;
    __syncthreads();
    for (int w = 1; w < 1024; w <<= 1) {  // inclusive Hillis-Steele scan
      const int v = t >= w ? sc[t - w] : 0;
      __syncthreads();
      sc[t] += v;
      __syncthreads();
    }
    int pos = (int)G + carry + sc[t] - n;
    if (gi < G)
      for (int f = 0; f < T; ++f)
        if ((m >> f) & 1u) {
          const int64_t q = gi * T + f;
          vpos[q] = pos;
          rows[pos] = (int)q;
          ++pos;
        }
    carry += sc[1023];
    __syncthreads();
  }
  if (t == 0) {
    stats[0] = carry;
    stats[1] = 0;
  }
}

// Exact values of the kept fingertips from the refine pass's stripe partials, then the group's
// first maximum of log(100·std) — the level kernel's choice — as the ∇std row: sel = its query,
// Xg = its point, vrow = its V row (list position).  stats[1] counts kept rows whose screen value
// missed the exact one by more than Δ (the calibration bound; 0 expected).
template <int KT>
__global__ __launch_bounds__(256) void refine_select_kernel(cdx_gpis g, const double* __restrict__ rpartial,
                                                            int64_t M_pad, int Nt, int64_t G, int T,
                                                            const double* __restrict__ sv2, const int* __restrict__ vpos,
                                                            const double* __restrict__ X, double* __restrict__ std_,
                                                            double* __restrict__ var, int64_t* __restrict__ sel,
                                                            double* __restrict__ Xg, int64_t* __restrict__ vrow,
                                                            int* __restrict__ stats) {
  const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= G) return;
  const double k0 = cdx::gpis_k0<KT>(g.R), delta = g.screen_delta;
  int fmax = 0;
  double lmax = 0;
  for (int f = 0; f < T; ++f) {
    const int64_t q = gi * T + f;
    const int pos = vpos[q];
    double sd;
    if (pos >= 0) {
      double acc = 0;
      for (int t = 0; t < Nt; ++t) acc += rpartial[(int64_t)t * M_pad + pos];
      const double v = k0 - acc;
      sd = sqrt(fabs(v));
      std_[q] = sd;
      var[q] = v;
      if (!(fabs(sv2[q] - v) <= delta) && isfinite(v)) atomicAdd(&stats[1], 1);
    } else {
      sd = std_[q];
    }
    const double lv = log(100 * sd);
    if (f == 0 || lv > lmax) { lmax = lv; fmax = f; }
  }
  const int64_t qi = gi * T + fmax;
  sel[gi] = qi;
  vrow[gi] = vpos[qi];
  for (int i = 0; i < 3; ++i) Xg[3 * gi + i] = X[3 * qi + i];
}

// ------------------------------------------------------------------ preparation (once per state)
// Centre of the inducing points (mean of rows < N, one block, fixed-order tree reduction) and the
// centred fp32 copy X1f [N_pad] (padding rows = row 0).
__global__ __launch_bounds__(256) void screen_center_kernel(cdx_gpis g, double* __restrict__ center,
                                                            float4* __restrict__ X1f) {
  __shared__ double red[3][256];
  const int t = threadIdx.x;
  double s[3] = {0, 0, 0};
  for (int j = t; j < g.N; j += 256)
    for (int c = 0; c < 3; ++c) s[c] += g.X1[3 * j + c];
  for (int c = 0; c < 3; ++c) red[c][t] = s[c];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w)
      for (int c = 0; c < 3; ++c) red[c][t] += red[c][t + w];
    __syncthreads();
  }
  const double cx = red[0][0] / g.N, cy = red[1][0] / g.N, cz = red[2][0] / g.N;
  if (t == 0) { center[0] = cx; center[1] = cy; center[2] = cz; center[3] = 0.0; }
  for (int j = t; j < g.N_pad; j += 256) {
    const int src = j < g.N ? j : 0;
    X1f[j] = make_float4((float)(g.X1[3 * src] - cx), (float)(g.X1[3 * src + 1] - cy), (float)(g.X1[3 * src + 2] - cz),
                         0.f);
  }
}

// L [N_pad/16][3][2][N_pad][8] bf16: slice s of L⁻ᵀ[16kb + 8h + e][j − shift] (zero for j < shift),
// the B-operand image the screen stages with one 16-byte load per (slice, k-half, column).
__global__ __launch_bounds__(256) void screen_split_kernel(cdx_gpis g, bf16x8* __restrict__ L) {
  const int Np = g.N_pad, shift = cdx::screen_shift(g.N, Np);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)(Np / 16) * 2 * Np) return;
  const int col = (int)(t % Np);
  const int h = (int)((t / Np) % 2);
  const int kb = (int)(t / (2 * (int64_t)Np));
  bf16x8 o[3];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int n = 16 * kb + 8 * h + e, j = col - shift;
    const double x = j >= 0 ? g.Linv_t[(int64_t)n * Np + j] : 0.0;
    const __bf16 a = (__bf16)(float)x;  // f64 → f32 → bf16: the f32 step keeps the split exact
    const double r1 = x - (double)(float)a;
    const __bf16 b = (__bf16)(float)r1;
    const double r2 = r1 - (double)(float)b;
    o[0][e] = a;
    o[1][e] = b;
    o[2][e] = (__bf16)(float)r2;
  }
  for (int s = 0; s < 3; ++s) L[(((int64_t)kb * 3 + s) * 2 + h) * Np + col] = o[s];
}

// csum[j] = k0 · Σ_{n<N} L⁻ᵀ[n][j − shift] (zero for j < shift): Ṽ = Ã·L⁻ᵀ + csum.  One 1024-thread
// block per 64 columns: 16 row groups each sum every 16th row, then a fixed-order combine.
template <int KT>
__global__ __launch_bounds__(1024) void screen_csum_kernel(cdx_gpis g, double* __restrict__ csum) {
  __shared__ double part[16][64];
  const int Np = g.N_pad, shift = cdx::screen_shift(g.N, Np);
  const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c, j = col - shift;
  double s = 0;
  if (j >= 0)
    for (int n = rg; n < g.N; n += 16) s += g.Linv_t[(int64_t)n * Np + j];
  part[rg][c] = s;
  __syncthreads();
  if (rg == 0) {
    double t = 0;
    for (int r = 0; r < 16; ++r) t += part[r][c];
    csum[col] = cdx::gpis_k0<KT>(g.R) * t;
  }
}

int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

}  // namespace

namespace cdx {

size_t screen_ws_bytes(const cdx_gpis& g, int64_t M) {
  return (size_t)(g.N_pad / SC_BN) * (size_t)round_up(M, SC_BM) * sizeof(double);
}

int screen_var_launch(const cdx_gpis& g, const double* X, int64_t M, double* var, void* ws, hipStream_t s) {
  if (M <= 0) return CDX_OK;
  const int64_t M_pad = round_up(M, SC_BM);
  const int Nt = g.N_pad / SC_BN;
  if (M_pad / SC_BM * Nt > 0x7fffffff) return CDX_EINVAL;
  const int Mt = (int)(M_pad / SC_BM);
  double* partial = static_cast<double*>(ws);
  const dim3 grid((unsigned)(Mt * Nt)), fgrid((unsigned)((M + 255) / 256));
  switch (g.kernel) {
    case CDX_KERNEL_TPS:
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_TPS>, grid, dim3(SC_THREADS), 0, s, g, X, M, partial, M_pad, Mt, Nt);
      hipLaunchKernelGGL(gpis_screen_finalize<CDX_KERNEL_TPS>, fgrid, dim3(256), 0, s, g, partial, M, M_pad, Nt, var);
      break;
    case CDX_KERNEL_RBF:
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_RBF>, grid, dim3(SC_THREADS), 0, s, g, X, M, partial, M_pad, Mt, Nt);
      hipLaunchKernelGGL(gpis_screen_finalize<CDX_KERNEL_RBF>, fgrid, dim3(256), 0, s, g, partial, M, M_pad, Nt, var);
      break;
    default:
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_JOINT>, grid, dim3(SC_THREADS), 0, s, g, X, M, partial, M_pad, Mt, Nt);
      hipLaunchKernelGGL(gpis_screen_finalize<CDX_KERNEL_JOINT>, fgrid, dim3(256), 0, s, g, partial, M, M_pad, Nt, var);
      break;
  }
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

size_t screen_select_ws_bytes(const cdx_gpis& g, int64_t Ms) { return screen_ws_bytes(g, Ms); }

int screen_select_launch(const cdx_gpis& g, const double* X, int64_t G, int T, void* ws, double* sv2, double* std_,
                         int* vpos, int* rows, unsigned char* keep, int* stats, hipStream_t s) {
  const int64_t Ms = G * T;
  if (G <= 0 || T <= 0 || T > CDX_MAX_TIPS) return CDX_EINVAL;
  const int64_t M_pad = round_up(Ms, SC_BM);
  const int Nt = g.N_pad / SC_BN;
  if (M_pad / SC_BM * Nt > 0x7fffffff || Ms > 0x7fffffff) return CDX_EINVAL;
  const int Mt = (int)(M_pad / SC_BM);
  double* partial = static_cast<double*>(ws);
  const dim3 grid((unsigned)(Mt * Nt)), sgrid((unsigned)((G + 255) / 256));
  switch (g.kernel) {
    case CDX_KERNEL_TPS:
      prof_mark(PROF_SCREEN, true, s);
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_TPS>, grid, dim3(SC_THREADS), 0, s, g, X, Ms, partial, M_pad, Mt, Nt);
      prof_mark(PROF_SCREEN, false, s);
      hipLaunchKernelGGL(screen_select_kernel<CDX_KERNEL_TPS>, sgrid, dim3(256), 0, s, g, partial, M_pad, Nt, G, T, sv2, std_, vpos, rows, keep);
      break;
    case CDX_KERNEL_RBF:
      prof_mark(PROF_SCREEN, true, s);
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_RBF>, grid, dim3(SC_THREADS), 0, s, g, X, Ms, partial, M_pad, Mt, Nt);
      prof_mark(PROF_SCREEN, false, s);
      hipLaunchKernelGGL(screen_select_kernel<CDX_KERNEL_RBF>, sgrid, dim3(256), 0, s, g, partial, M_pad, Nt, G, T, sv2, std_, vpos, rows, keep);
      break;
    default:
      prof_mark(PROF_SCREEN, true, s);
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_JOINT>, grid, dim3(SC_THREADS), 0, s, g, X, Ms, partial, M_pad, Mt, Nt);
      prof_mark(PROF_SCREEN, false, s);
      hipLaunchKernelGGL(screen_select_kernel<CDX_KERNEL_JOINT>, sgrid, dim3(256), 0, s, g, partial, M_pad, Nt, G, T, sv2, std_, vpos, rows, keep);
      break;
  }
  hipLaunchKernelGGL(screen_compact_kernel, dim3(1), dim3(1024), 0, s, G, T, (const unsigned char*)keep, vpos, rows, stats);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int refine_select_launch(const cdx_gpis& g, const double* X, int64_t G, int T, const double* rpartial, int64_t M_pad,
                         const double* sv2, const int* vpos, double* std_, double* var, int64_t* sel, double* Xg,
                         int64_t* vrow, int* stats, hipStream_t s) {
  const int Nt = g.N_pad / SC_BN;
  const dim3 sgrid((unsigned)((G + 255) / 256));
  switch (g.kernel) {
    case CDX_KERNEL_TPS:
      hipLaunchKernelGGL(refine_select_kernel<CDX_KERNEL_TPS>, sgrid, dim3(256), 0, s, g, rpartial, M_pad, Nt, G, T, sv2, vpos, X, std_, var, sel, Xg, vrow, stats);
      break;
    case CDX_KERNEL_RBF:
      hipLaunchKernelGGL(refine_select_kernel<CDX_KERNEL_RBF>, sgrid, dim3(256), 0, s, g, rpartial, M_pad, Nt, G, T, sv2, vpos, X, std_, var, sel, Xg, vrow, stats);
      break;
    default:
      hipLaunchKernelGGL(refine_select_kernel<CDX_KERNEL_JOINT>, sgrid, dim3(256), 0, s, g, rpartial, M_pad, Nt, G, T, sv2, vpos, X, std_, var, sel, Xg, vrow, stats);
      break;
  }
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

}  // namespace cdx

extern "C" {

size_t cdx_gpis_screen_bytes(int32_t N_pad) {
  if (N_pad <= 0 || N_pad % CDX_NPAD_ALIGN) return 0;
  return cdx::screen_bytes(N_pad);
}

int cdx_gpis_screen_prepare(const cdx_gpis* g, void* screen, cdx_stream_t stream) {
  if (!g || !g->X1 || !g->Linv_t || !screen || g->N <= 0 || g->N_pad < g->N || g->N_pad % CDX_NPAD_ALIGN) return CDX_EINVAL;
  if (g->kernel < 0 || g->kernel > 2) return CDX_EKERNEL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  cdx_gpis gv = *g;
  gv.screen = screen;
  const cdx::ScreenView v = cdx::screen_view(gv);
  const int Np = g->N_pad;
  hipLaunchKernelGGL(screen_center_kernel, dim3(1), dim3(256), 0, s, gv, const_cast<double*>(v.center),
                     const_cast<float4*>(v.X1f));
  const int64_t nsplit = (int64_t)(Np / 16) * 2 * Np;
  hipLaunchKernelGGL(screen_split_kernel, dim3((unsigned)((nsplit + 255) / 256)), dim3(256), 0, s, gv,
                     reinterpret_cast<bf16x8*>(const_cast<void*>(v.L)));
  const dim3 cgrid((unsigned)(Np / 64)), cblk(1024);
  switch (g->kernel) {
    case CDX_KERNEL_TPS: hipLaunchKernelGGL(screen_csum_kernel<CDX_KERNEL_TPS>, cgrid, cblk, 0, s, gv, const_cast<double*>(v.csum)); break;
    case CDX_KERNEL_RBF: hipLaunchKernelGGL(screen_csum_kernel<CDX_KERNEL_RBF>, cgrid, cblk, 0, s, gv, const_cast<double*>(v.csum)); break;
    default: hipLaunchKernelGGL(screen_csum_kernel<CDX_KERNEL_JOINT>, cgrid, cblk, 0, s, gv, const_cast<double*>(v.csum)); break;
  }
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

size_t cdx_gpis_screen_workspace(const cdx_gpis* g, int64_t M) {
  if (!g || M <= 0 || g->N_pad <= 0) return 0;
  return cdx::screen_ws_bytes(*g, M);
}

int cdx_gpis_screen_var(const cdx_gpis* g, const double* X, int64_t M, double* var, void* workspace,
                        cdx_stream_t stream) {
  if (!g || !g->screen || !g->X1 || g->N <= 0 || g->N_pad % CDX_NPAD_ALIGN) return CDX_EINVAL;
  if (g->kernel < 0 || g->kernel > 2) return CDX_EKERNEL;
  if (M < 0 || (M > 0 && (!X || !var || !workspace))) return CDX_EINVAL;
  return cdx::screen_var_launch(*g, X, M, var, workspace, reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
