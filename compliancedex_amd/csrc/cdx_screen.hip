// Split-precision screen of the GPIS posterior variance on the fp16 matrix cores (gfx950).
//
// The closure's variance cost reads only max_f log(100·std_f) over a candidate's fingertips
// (optimize_pregrasp.py:733): one fingertip per (level, candidate) reaches the loss and its
// gradient.  The screen estimates std² = k0 − ‖L⁻¹k‖² (gpis.py:56-59, whitened form) for every
// all-tip query at a fraction of the fp64 cost, so that the exact fp64 whitened pass only runs
// for the fingertips that can still be the maximum (cdx_closure, cdx_screen_select below):
//
//   Ṽ = Ã·L⁻ᵀ + k0·colsum(L⁻ᵀ),  Ã = K* − k0   (the offset keeps |Ã| small near the query, where
//                                              the cancellation in k0 − ‖V‖² is worst)
//   Ã (scaled by a power of two SA, k0·SA ≤ 2¹⁰) and L⁻ᵀ (column j scaled by a power of two SB_j,
//   max |column|·SB_j < 2¹⁴) are each split into two fp16 slices (x = x0 + x1, ≈ 22 bits), and the
//   three slice products of index sum ≤ 1 are accumulated into one fp32 accumulator per output by
//   v_mfma_f32_32x32x16_f16; the epilogue multiplies by 1/(SA·SB_j) (exact).  The error is set by
//   the fp32 generation and accumulation, not the 22-bit operands: the CPU emulation gives the same
//   1.5e-6·k0 as three bf16 slices with six products (round 2's first version), at half the MFMAs
//   and two thirds of the operand bytes.  Σ Ṽ² is summed in f64.  A query farther than rq from the
//   inducing points' centre (where SA·Ã could leave fp16's range) is made NaN, so the closure runs
//   the exact pass for its whole group.
//
// The estimate carries no parity claim by itself: the closure only uses it to discard fingertips
// whose estimated std² is below the leader's by more than twice the per-object error bound
// (cdx_gpis.screen_delta, calibrated against the fp64 pass when the state is built), and writes
// exact fp64 values for every fingertip it keeps.  tools/screen_emul.py emulates this arithmetic
// on the CPU (max |Δstd²|/k0 = 1.5e-6 on the config-2 workload).
#include <hip/hip_runtime.h>

#include "cdx_ab.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "cdx_gpis.h"
#include "cdx_gpis_launch.h"
#include "cdx_prof.h"
#include "cdx_screen.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

using cdx::SC_BK;
using cdx::SC_BN;
constexpr int SC_BM = 256;                 // query rows per workgroup
#ifndef CDX_SC_WAVES
#define CDX_SC_WAVES 8
#endif
// 8 waves (two per SIMD): 2 (rows) × 4 (columns), 128 × 64 outputs each; 4 waves (one per SIMD,
// accumulators in AGPRs): 2 × 2, 128 × 128 outputs each (half the fragment reads per MFMA);
// 16 waves (four per SIMD, ≤ 128 registers): 4 × 4, 64 × 64 outputs each
constexpr int SC_W = CDX_SC_WAVES;
static_assert(SC_W == 8 || SC_W == 4 || SC_W == 16, "4, 8 or 16 waves per workgroup");
constexpr int SC_THREADS = 64 * SC_W;
constexpr int SC_WC = SC_W == 4 ? 128 : 64;   // columns per wave
constexpr int SC_WR = SC_W == 16 ? 64 : 128;  // rows per wave
constexpr int SC_NJ = SC_WC / 32;             // 32-column accumulator blocks per wave
constexpr int SC_NI = SC_WR / 32;             // 32-row accumulator blocks per wave
constexpr int SC_GKH = SC_W == 4 ? 2 : 1;     // k-halves generated per thread per sub-step
// 16 waves: each thread generates one (sub-step, k-half) chunk of the next stage
constexpr int SC_REG = 4 * 256;            // 16-byte LDS units of one 16-K sub-step: [slice][khalf][256]
#ifndef CDX_SC_SUB
#define CDX_SC_SUB 2
#endif
constexpr int SC_SUB = CDX_SC_SUB;         // 16-K sub-steps per stage (one barrier per stage)
#ifndef CDX_SC_RING
#define CDX_SC_RING (CDX_SC_SUB == 1 ? 3 : 2)
#endif
constexpr int SC_RING = CDX_SC_RING;       // B stages in LDS: DMA'd SC_RING − 1 stages ahead
static_assert(SC_RING == 2 || SC_RING == 3, "B ring of 2 or 3 stages");
constexpr int SC_NDMA = 16 * SC_SUB / SC_W;  // 1-KB DMAs per wave per stage
static_assert(SC_SUB == 1 || SC_SUB == 2, "stage = 16 or 32 K rows");
#ifndef CDX_SC_PP
#define CDX_SC_PP 0
#endif
#ifndef CDX_SC_EPI_REG  // epilogue from the accumulator registers (1, default) or through an LDS image (0)
#define CDX_SC_EPI_REG 1
#endif
// Ping-pong: the two waves of a SIMD (waves w, w+4) multiply in alternate half-stages; in the
// other half each generates one 16-K sub-step of the next stage's A and DMAs its B.
constexpr bool SC_PP = CDX_SC_PP;
static_assert(!SC_PP || (SC_W == 8 && SC_SUB == 2 && SC_RING == 2), "ping-pong: 8 waves, 32-K stages, B ring of 2");
// Epilogue image of one row half of the tile: fp32 rows of pitch SC_LDE ≡ 4 (mod 32), the e-th
// 64-column share of a row rotated by 16·e dwords (sc_tcol): the accumulators' ds_write_b128 (8
// consecutive rows per lane group) and the summing threads' ds_read_b128 (4 shares × 4 rows per
// lane group) are both conflict-free.  Then the stripe's (cscale, csum) pairs, pair c at c + (c >> 6).
constexpr int SC_LDE = 260;
constexpr int SC_EPI_CF = 128 * SC_LDE * 4;
constexpr int SC_EPI = SC_EPI_CF + (SC_BN + SC_BN / 64) * 16;
// LDS: A stages (generated, 2 buffers) | B stages (LDS-DMA ring); after the loop, the epilogue
constexpr int SC_A_OFF = 0, SC_B_OFF = 2 * SC_SUB * SC_REG * 16;
constexpr int SC_SMEM = std::max(SC_B_OFF + SC_RING * SC_SUB * SC_REG * 16, SC_EPI);
static_assert(SC_SMEM <= 160 * 1024, "screen stage buffers exceed the CU's LDS");

// K-steps (16 rows of L⁻ᵀ) of stripe nt: rows [0, min(N, (nt+1)·256 − shift)) as in the fp64 pass.
__device__ __host__ inline int sc_ksteps(int nt, int N, int Np) {
  const int hi = std::min(N, (nt + 1) * SC_BN - cdx::screen_shift(N, Np));
  return (hi + SC_BK - 1) / SC_BK;
}

// SA·Ã = SA·(k(r) − k(0)) in fp32 from a centred fp32 offset (d = x − x_n); kc = {SA·w_rbf,
// 2·SA·w_tps, 3R·SA·w_tps, −0.5/σ²} with the joint kernel's weights w (0.3, 0.7) or 1.
template <int KT>
__device__ __forceinline__ float k_offset(float dx, float dy, float dz, const float4& kc) {
  const float r2 = dx * dx + dy * dy + dz * dz;
  if (KT == CDX_KERNEL_RBF) return kc.x * expm1f(r2 * kc.w);
  const float r = __builtin_amdgcn_sqrtf(r2);  // v_sqrt_f32 (≤ 1 ulp): ample for a screen
  const float tps = r2 * (kc.y * r - kc.z);    // SA·(2r³ − 3Rr²)  (= SA·(TPS − R³))
  if (KT == CDX_KERNEL_TPS) return tps;
  return kc.x * expm1f(r2 * kc.w) + tps;
}

// (xa, xb) = (a0 + a1, b0 + b1): fp16 pairs truncated from fp32 (v_cvt_pkrtz_f16_f32); the
// remainders x − x0 are exact in fp32, so the split loses only the second truncation (≤ 2⁻²⁰·|x|).
__device__ __forceinline__ void split2(float xa, float xb, unsigned& h0, unsigned& h1) {
  const auto p = __builtin_amdgcn_cvt_pkrtz(xa, xb);
  const auto q = __builtin_amdgcn_cvt_pkrtz(xa - (float)p[0], xb - (float)p[1]);
  h0 = __builtin_bit_cast(unsigned, p);
  h1 = __builtin_bit_cast(unsigned, q);
}

// One workgroup per (query tile of 256 rows, stripe of 256 columns); stripes paired heavy+light per
// XCD as in gpis_std_kernel<VAR>.  partial[nt][m] = Σ over the stripe's columns of (Ã·L⁻ᵀ + c)².
template <int KT>
__global__ __launch_bounds__(SC_THREADS, SC_W / 4) void gpis_screen_kernel(cdx_gpis g, const double* __restrict__ X, int64_t M,
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
  const int nK = sc_ksteps(nt, N, Np);        // 16-K sub-steps
  const int nS = (nK + SC_SUB - 1) / SC_SUB;  // stages

  // generation: thread → query row grow, k-halves gkh .. gkh + SC_GKH − 1 (wave-uniform), 8 entries each
  const int grow = tid & (SC_BM - 1);
  const int gkh = SC_W == 4 ? 0 : __builtin_amdgcn_readfirstlane((tid >> 8) & 1);
  const int gsub = SC_W == 16 ? __builtin_amdgcn_readfirstlane(tid >> 9) : 0;
  float qx, qy, qz;
  {
    const int64_t m = std::min(m0 + grow, M - 1);  // pad rows replicate a valid query
    qx = (float)(X[3 * m] - sv.center[0]);
    qy = (float)(X[3 * m + 1] - sv.center[1]);
    qz = (float)(X[3 * m + 2] - sv.center[2]);
    if (!(qx * qx + qy * qy + qz * qz <= (float)sv.center[4])) qx = __builtin_nanf("");  // SA·Ã may overflow fp16
  }
  float4 kc;
  {
    const double SA = sv.center[3], w = KT == CDX_KERNEL_JOINT ? 0.7 : 1.0;
    kc = make_float4((float)(SA * (KT == CDX_KERNEL_JOINT ? 0.3 : 1.0)), (float)(2.0 * SA * w), (float)(3.0 * g.R * SA * w),
                     (float)(-0.5 / (g.sigma * g.sigma)));
  }

  // wave → 128 × SC_WC output sub-tile; with 8 waves, waves w and w+4 share a SIMD and take
  // complementary columns
  // (16 waves: waves w, w+4, w+8, w+12 share a SIMD and take all four column quarters)
  const int cwave = SC_W == 16 ? (((wave & 3) + (wave >> 2)) & 3) : SC_W == 8 ? (wave < 4 ? wave : 7 - wave) : (wave & 1);
  const int wr = (SC_W == 16 ? (wave >> 2) : SC_W == 8 ? (wave >> 2) : (wave >> 1)) * SC_WR;
  const int wc = cwave * SC_WC;
  // B rows past this wave's last column are zero (upper-triangular L⁻ᵀ, shifted columns)
  const int kend_w = __builtin_amdgcn_readfirstlane(n0 + wc + SC_WC - shift);

  f32x16 acc[SC_NI][SC_NJ];
#pragma unroll
  for (int i = 0; i < SC_NI; ++i)
#pragma unroll
    for (int j = 0; j < SC_NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Staging by LDS-DMA (global_load_lds: no VGPRs, no ds_write).  issue(st): every wave DMAs
  // SC_NDMA × 1 KB of B stage st (instruction u = wave + 8i: sub-step u>>4, slice/k-half region
  // (u>>2)&3, columns 64·(u&3) + lane) into ring slot st % SC_RING, SC_RING − 1 stages ahead.
  // 32-K stages (default): issue(s+1) during step s, `s_waitcnt vmcnt(0)` before the step's raw
  // s_barrier.  16-K stages: issue(s+2) during step s and a counted `vmcnt(2)` keeps that step's DMAs
  // in flight across the barrier (__syncthreads would wait vmcnt(0)); clamped stages past the
  // stripe's end load into free slots, so every step issues the same count.
  const char* Lb = static_cast<const char*>(sv.L);
  auto issue = [&](int st) {
    const int sc = std::min(st, nS - 1);
    const int slot = st % SC_RING;
#if defined(CDX_SC_DIAG_NODMA)  // timing-only diagnostic build: outputs are wrong
    if (st > 0) return;
#endif
#pragma unroll
    for (int i = 0; i < SC_NDMA; ++i) {
      const int u = wave + SC_W * i, sub = u >> 4, r = u & 15, col = 64 * (r & 3) + lane;
      const char* src = Lb + (((int64_t)((sc * SC_SUB + sub) * 4 + (r >> 2))) * Np + n0 + col) * 16;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sB4 + (slot * SC_SUB + sub) * SC_REG + r * 64),
                                       16, 0, 0);
    }
  };
  u32x4 ast[2];      // generated A sub-step: 8 entries × 2 fp16 slices, packed in pairs
  // X1 rows of the generated stage: wave-uniform addresses → scalar loads (SMEM; the vector memory
  // counter stays free for the DMAs' counted waits)
  auto gen_a = [&](int st, int sub, int kh) {  // 8 consecutive k of k-half kh, packed in pairs
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float4 cfloat4;  // constant space: SMEM loads
#else
    typedef const float4 cfloat4;
#endif
    cfloat4* x1 = (cfloat4*)(sv.X1f) + __builtin_amdgcn_readfirstlane((st * SC_SUB + sub) * SC_BK + 8 * kh);
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const float4 p = x1[e], p1 = x1[e + 1];
      unsigned h0, h1;
#if defined(CDX_SC_DIAG_NOGEN)  // timing-only diagnostic build: outputs are wrong
      split2(qx - p.x, qy - p1.y, h0, h1);
#else
      split2(k_offset<KT>(qx - p.x, qy - p.y, qz - p.z, kc), k_offset<KT>(qx - p1.x, qy - p1.y, qz - p1.z, kc), h0, h1);
#endif
      ast[0][e / 2] = h0;
      ast[1][e / 2] = h1;
    }
  };
  auto write_a = [&](int buf, int sub, int kh) {
#pragma unroll
    for (int i = 0; i < 2; ++i) sA4[(buf * SC_SUB + sub) * SC_REG + (i * 2 + kh) * 256 + grow] = ast[i];
  };
  auto gen_write = [&](int st, int buf, int sub) {
#pragma unroll
    for (int h = 0; h < SC_GKH; ++h) {
      gen_a(st, sub, gkh + h);
      write_a(buf, sub, gkh + h);
    }
  };
  // one sub-step's 12·SC_NJ MFMAs: lane → (row/col l&31, k-half l>>5); B slices of the wave's column
  // blocks, A slice by slice (products of slice-index sum ≤ 1, smallest first); each MFMA takes the
  // B slice as its A operand (Ṽᵀ blocks: see the epilogue)
  auto mfma_sub = [&](int abuf, int bslot, int sub, auto more_c) {
    constexpr bool MORE = decltype(more_c)::value;
    const u32x4* a4 = sA4 + (abuf * SC_SUB + sub) * SC_REG;
    const u32x4* b4 = sB4 + (bslot * SC_SUB + sub) * SC_REG;
    f16x8 fb[2][SC_NJ];
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int j = 0; j < SC_NJ; ++j)
#if defined(CDX_SC_DIAG_NOREAD)  // timing-only diagnostic build: outputs are wrong
        fb[sb][j] = __builtin_bit_cast(f16x8, u32x4{(unsigned)lane, (unsigned)j, (unsigned)sb, (unsigned)sub});
#else
        fb[sb][j] = __builtin_bit_cast(f16x8, b4[(sb * 2 + (lane >> 5)) * 256 + wc + 32 * j + (lane & 31)]);
#endif
#pragma unroll
    for (int sa = 1; sa >= 0; --sa) {
      f16x8 fa[SC_NI];
#pragma unroll
      for (int i = 0; i < SC_NI; ++i)
#if defined(CDX_SC_DIAG_NOREAD)
        fa[i] = __builtin_bit_cast(f16x8, u32x4{(unsigned)lane, (unsigned)i, (unsigned)sa, (unsigned)abuf});
#else
        fa[i] = __builtin_bit_cast(f16x8, a4[(sa * 2 + (lane >> 5)) * 256 + wr + 32 * i + (lane & 31)]);
#endif
#pragma unroll
      for (int sb = 1 - sa; sb >= 0; --sb)
#pragma unroll
        for (int i = 0; i < SC_NI; ++i)
#pragma unroll
          for (int j = 0; j < SC_NJ; ++j)
#if defined(CDX_SC_DIAG_NOMFMA)  // timing-only diagnostic build: outputs are wrong
            acc[i][j][0] += (float)fa[i][0] * (float)fb[sb][j][0];
#else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[sb][j], fa[i], acc[i][j], 0, 0, 0);
#endif
      if (!MORE) __builtin_amdgcn_sched_barrier(0);  // tail step: no fragment hoisting past a slice group
    }
  };

#if defined(CDX_SC_PRIO_YOUNG)  // A/B: static priority for the second-dispatched half (waves 4–7)
  if (wave >= SC_W / 2) __builtin_amdgcn_s_setprio(1);
#endif
  // prologue: B stages 0 .. SC_RING−2 landed, A of stage 0 generated
#pragma unroll
  for (int st = 0; st < SC_RING - 1; ++st) issue(st);
  if constexpr (SC_W == 16) {
    gen_a(0, gsub, gkh);
    write_a(0, gsub, gkh);
  } else {
#pragma unroll
    for (int u = 0; u < SC_SUB; ++u) gen_write(0, 0, u);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // Step s multiplies stage s (A buffer s&1, B slot s % SC_RING) while stage s + SC_RING − 1 is DMA'd
  // and stage s+1's A is generated and written to the other A buffer, sub-step by sub-step.  NLIVE:
  // this wave's B columns are non-zero in the first NLIVE sub-steps of stage s; MORE: a stage s+1
  // exists.  Each (NLIVE, MORE) body is one straight-line block, so the generation's VALU work
  // interleaves with the MFMAs.
  auto step = [&](int s, auto nlive_c, auto more_c) {
    constexpr int NLIVE = decltype(nlive_c)::value;
    constexpr bool MORE = decltype(more_c)::value;
    if (SC_RING > 2 || s + 1 < nS) issue(s + SC_RING - 1);
#pragma unroll
    for (int u = 0; u < SC_SUB; ++u) {
      if constexpr (SC_W == 16) {
        if (MORE && u == 0) gen_a(s + 1, gsub, gkh);
        if (u < NLIVE) mfma_sub(s & 1, s % SC_RING, u, more_c);
        if (MORE && u == 0) write_a((s + 1) & 1, gsub, gkh);
      } else if (SC_GKH == 1) {
        if (MORE) gen_a(s + 1, u, gkh);
        if (u < NLIVE) mfma_sub(s & 1, s % SC_RING, u, more_c);
        if (MORE) write_a((s + 1) & 1, u, gkh);
      } else {
        if (u < NLIVE) mfma_sub(s & 1, s % SC_RING, u, more_c);
        if (MORE) gen_write(s + 1, (s + 1) & 1, u);
      }
    }
    // B stage s+1 landed (the newest stage's DMAs may stay in flight), A written
    if constexpr (SC_RING == 2)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else if constexpr (SC_NDMA == 2)
      asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
#if !defined(CDX_SC_DIAG_NOBAR)  // timing-only diagnostic build (races): outputs are wrong
    __builtin_amdgcn_s_barrier();
#endif
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const int k_live = std::min(nK, std::max(0, (kend_w + SC_BK - 1) / SC_BK));  // live sub-steps (wave-uniform)
  if constexpr (SC_PP) {
    // Phase ph of stage s: waves 0–3 (ph 0) or 4–7 (ph 1) multiply stage s; the other half DMAs
    // sub-step ph of B(s+1) (4 KB per wave) and generates sub-step ph of A(s+1) (both k-halves of
    // its 256 rows).  Buffers: A(s+1) and B(s+1) go to the slots stage s−1 used, free since the
    // barrier that ended stage s−1; B(s+1) has landed at the barrier that ends stage s.
    const bool P = wave < 4;
    for (int s = 0; s < nS; ++s) {
      const bool more = s + 1 < nS;
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        if (P == (ph == 0)) {
          if (2 * s < k_live) mfma_sub(s & 1, s % SC_RING, 0, T_{});
          if (2 * s + 1 < k_live) mfma_sub(s & 1, s % SC_RING, 1, T_{});
        } else if (more) {
          const int sc = s + 1, slot = sc % SC_RING;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = (wave & 3) + 4 * i, col = 64 * (r & 3) + lane;
            const char* src = Lb + (((int64_t)((sc * SC_SUB + ph) * 4 + (r >> 2))) * Np + n0 + col) * 16;
            __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sB4 + (slot * SC_SUB + ph) * SC_REG + r * 64),
                                             16, 0, 0);
          }
#pragma unroll
          for (int kh = 0; kh < 2; ++kh) {
            gen_a(sc, ph, kh);
            write_a(sc & 1, ph, kh);
          }
        }
        if (ph == 0)
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
  } else {
    const int full = k_live / SC_SUB;
    int s = 0;
    for (; s < std::min(full, nS - 1); ++s) step(s, std::integral_constant<int, SC_SUB>{}, T_{});
    if (SC_SUB == 2 && s < nS - 1 && s * SC_SUB < k_live) {
      step(s, std::integral_constant<int, 1>{}, T_{});
      ++s;
    }
    for (; s < nS - 1; ++s) step(s, std::integral_constant<int, 0>{}, T_{});
    // last stage: its MFMAs only; then every DMA drained before the epilogue reuses the LDS
#pragma unroll
    for (int u = 0; u < SC_SUB; ++u)
      if (s * SC_SUB + u < k_live) mfma_sub(s & 1, s % SC_RING, u, F_{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Epilogue: per row Σ over the stripe's 256 columns of (Ṽ + c)² in f64.  The MFMAs compute Ṽᵀ (L⁻ᵀ
  // slice as the A operand, Ã as B), so reg r of lane l holds query row l&31, column (r&3) + 8(r>>2) +
  // 4(l>>5).  Default (CDX_SC_EPI_REG=1): each lane sums its own columns straight from the accumulators
  // into one f64 per row block (below; 0.175 vs 0.181 ms per screen in the closure, standalone 0.207–0.211
  // vs 0.218 ms against 0.200–0.204 with no epilogue at all, profiles/r03u_screen_epilogue_ab.jsonl).
  // CDX_SC_EPI_REG=0: the accumulators go through LDS one row half at a time (four consecutive columns
  // per register quad, one ds_write_b128, rotated conflict-free image), then EP threads per row sum a
  // share of its columns each, in column order, and combine by xor-shuffles.  Both stage the columns'
  // (cscale, csum) in LDS once (read from global memory per thread, they cost a quarter of the kernel).
#if defined(CDX_SC_DIAG_NOEPI)  // timing-only diagnostic build: outputs are wrong
  {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < SC_NI; ++i)
#pragma unroll
      for (int j = 0; j < SC_NJ; ++j) t += acc[i][j][0] + acc[i][j][15];
    if (lane == 0) partial[(int64_t)nt * M_pad + m0 + wave] = t;
    return;
  }
#endif
#if CDX_SC_EPI_REG
  // Register epilogue: each lane sums (Ṽ·cscale + csum)² over its own 32 columns of its rows straight
  // from the accumulators (columns in (j, r) order, the (cscale, csum) pairs broadcast from LDS), the
  // two column halves of a lane pair combine by one xor-shuffle, and the column waves of a row through
  // LDS in column-wave order — no accumulator image in LDS and one barrier instead of three.
  {
    double2* CF = reinterpret_cast<double2*>(smem);                          // [SC_BN] (cscale, csum)
    double* red = reinterpret_cast<double*>(smem + SC_BN * sizeof(double2));  // [SC_BN / SC_WC][SC_BM]
    if (tid < SC_BN) CF[tid] = make_double2(sv.cscale[n0 + tid], sv.csum[n0 + tid]);
    __syncthreads();
    double sum[SC_NI];
#pragma unroll
    for (int i = 0; i < SC_NI; ++i) sum[i] = 0.0;
#pragma unroll
    for (int j = 0; j < SC_NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const double2 cf = CF[wc + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)];
#pragma unroll
        for (int i = 0; i < SC_NI; ++i) {
          const double x = fma((double)acc[i][j][r], cf.x, cf.y);
          sum[i] = fma(x, x, sum[i]);
        }
      }
#pragma unroll
    for (int i = 0; i < SC_NI; ++i) {
      sum[i] += __shfl_xor(sum[i], 32);
      if (lane < 32) red[cwave * SC_BM + wr + 32 * i + lane] = sum[i];
    }
    __syncthreads();
    if (tid < SC_BM) {
      double t = 0.0;
#pragma unroll
      for (int c = 0; c < SC_BN / SC_WC; ++c) t += red[c * SC_BM + tid];
      partial[(int64_t)nt * M_pad + m0 + tid] = t;
    }
    return;
  }
#endif
  float* T = reinterpret_cast<float*>(smem);
  double2* CF = reinterpret_cast<double2*>(smem + SC_EPI_CF);
  constexpr int EP = SC_W == 4 ? 2 : 4, ECOL = SC_BN / EP;  // threads per row, columns per thread
  const int erow = tid / EP, epart = tid % EP;
  auto tcol = [](int c) { return (c & ~63) + (((c & 63) + 16 * (c >> 6)) & 63); };
  if (tid < SC_BN) CF[tid + (tid >> 6)] = make_double2(sv.cscale[n0 + tid], sv.csum[n0 + tid]);
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    if (ph) __syncthreads();  // phase 0's readers are done with T
    if ((wr >> 7) == ph) {
#pragma unroll
      for (int i = 0; i < SC_NI; ++i)
#pragma unroll
        for (int j = 0; j < SC_NJ; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<float4*>(T + ((wr & 127) + 32 * i + (lane & 31)) * SC_LDE + tcol(wc + 32 * j + 8 * q + 4 * (lane >> 5))) =
                make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
    }
    __syncthreads();
    if (tid < 128 * EP) {  // 16 waves: the first 8 sum (the same column split and order)
      const float* Tr = T + erow * SC_LDE;
      double sum = 0.0;
#pragma unroll 4
      for (int c = 0; c < ECOL / 4; ++c) {
        const int c0 = ECOL * epart + 4 * c;  // 4 columns inside one 64-column share
        const float4 v = *reinterpret_cast<const float4*>(Tr + tcol(c0));
        const double2* p = CF + c0 + (c0 >> 6);
        const double2 p0 = p[0], p1 = p[1], p2 = p[2], p3 = p[3];
        const double x0 = fma((double)v.x, p0.x, p0.y), x1 = fma((double)v.y, p1.x, p1.y),
                     x2 = fma((double)v.z, p2.x, p2.y), x3 = fma((double)v.w, p3.x, p3.y);
        sum = fma(x0, x0, sum);
        sum = fma(x1, x1, sum);
        sum = fma(x2, x2, sum);
        sum = fma(x3, x3, sum);
      }
#pragma unroll
      for (int w = 1; w < EP; w <<= 1) sum += __shfl_xor(sum, w);
      if (epart == 0) partial[(int64_t)nt * M_pad + m0 + 128 * ph + erow] = sum;
    }
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
// takes max_f log(100·std_f) over a group (optimize_pregrasp.py:733) with std = sqrt(|var|)
// (gpis.py:59).  Per group: s̃²_f = k0 − Σ stripe partials, a_f = |s̃²_f| with the row's margin
// Δ_f = Δ·max(1, (k0 − s̃²_f)/k0) (Δ = g.screen_delta, calibrated so |s̃² − var| ≤ Δ_f; the factor is
// ‖Ṽ‖²/k0, the scale of the estimate's rounding, 1 near the object), so |var_f| ∈ [a_f − Δ_f, a_f +
// Δ_f].  Leader = first maximum of a_f; kept for the exact pass: every f with a_f + Δ_f ≥ max_g (a_g
// − Δ_g) (the leader always), all T when a value is not finite.  A discarded fingertip gets std =
// sqrt(a_f), below the exact std of the group's maximum, so the level kernel's argmax is unchanged.
// The per-group selection kernels (one thread per group, latency-bound loads of the stripe partials)
// run in 64-thread workgroups: G = 4096 groups spread over 64 CUs instead of 16.
constexpr int SEL_BLOCK = cdx::SCREEN_SEL_BLOCK;  // (screen_compact_words sizes the histograms from it)

using cdx::screen_margin;

// Per group: estimates, leader, kept rows, and each discarded row's normalised gap z (cdx_screen.h) for
// the audit, which the compaction kernel picks: the discarded rows nearest the keep threshold.  A
// function of the inputs only: the same inputs give the same exact-pass list, hence bit-identical results
// (the refine pass's K-split depends on the list length).
template <int KT>
__device__ __forceinline__ void select_group(const cdx_gpis& g, const double* __restrict__ partial, int64_t M_pad, int Nt,
                                             int64_t gi, int T, double* __restrict__ sv2, double* __restrict__ std_,
                                             int* __restrict__ vpos, int* __restrict__ rows,
                                             unsigned short* __restrict__ keep, unsigned* __restrict__ zkey,
                                             const double* __restrict__ X, int* s_hist) {
  const double k0 = cdx::gpis_k0<KT>(g.R), delta = g.screen_delta;
  const double* ctr = cdx::screen_view(g).center;
  double a[CDX_MAX_TIPS], d[CDX_MAX_TIPS];
  bool finite = true;
  int lead = 0;
  double lo = -INFINITY;
  for (int f = 0; f < T; ++f) {
    const int64_t q = gi * T + f;
    double acc = 0;
    for (int t = 0; t < Nt; ++t) acc += partial[(int64_t)t * M_pad + q];
    const double s2 = k0 - acc;
    sv2[q] = s2;
    a[f] = fabs(s2);
    d[f] = screen_margin(delta, ctr, cdx::screen_band(ctr, X[3 * q], X[3 * q + 1], X[3 * q + 2]), k0, s2);
    finite = finite && isfinite(s2) && isfinite(d[f]);
    if (a[f] > a[lead]) lead = f;
    lo = fmax(lo, a[f] - d[f]);
  }
  unsigned mask = 0;
  for (int f = 0; f < T; ++f) {
    const int64_t q = gi * T + f;
    unsigned z = cdx::Z_NONE;
    if (f == lead) {
      vpos[q] = (int)gi;
      rows[gi] = (int)q;
    } else if (!finite || a[f] + d[f] >= lo) {
      mask |= 1u << f;  // kept: position assigned by screen_place_kernel
    } else {
      vpos[q] = -1;  // discarded (the compaction may still list it as audited)
      std_[q] = sqrt(a[f]);
      z = __float_as_uint((float)((lo - a[f]) / d[f]));
      atomicAdd(&s_hist[cdx::audit_bin(z)], 1);
    }
    zkey[q] = z;
  }
  keep[gi] = (unsigned short)mask;
}

// The select kernel also writes its block's histogram of the discarded rows' z bins (one row of AUDIT_BINS ints
// per block, fully overwritten: no zeroing between closures) for the compaction's audit cut.
template <int KT>
__global__ __launch_bounds__(SEL_BLOCK) void screen_select_kernel(cdx_gpis g, const double* __restrict__ partial,
                                                                  int64_t M_pad, int Nt, int64_t G, int T,
                                                                  double* __restrict__ sv2, double* __restrict__ std_,
                                                                  int* __restrict__ vpos, int* __restrict__ rows,
                                                                  unsigned short* __restrict__ keep,
                                                                  unsigned* __restrict__ zkey, const double* __restrict__ X,
                                                                  int* __restrict__ hist) {
  __shared__ int s_hist[cdx::AUDIT_BINS];
  for (int i = threadIdx.x; i < cdx::AUDIT_BINS; i += SEL_BLOCK) s_hist[i] = 0;
  __syncthreads();
  const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gi < G) select_group<KT>(g, partial, M_pad, Nt, gi, T, sv2, std_, vpos, rows, keep, zkey, X, s_hist);
  __syncthreads();
  for (int i = threadIdx.x; i < cdx::AUDIT_BINS; i += SEL_BLOCK) hist[(int64_t)blockIdx.x * cdx::AUDIT_BINS + i] = s_hist[i];
}

// Deterministic compaction of the kept non-leader fingertips and the audited rows behind the G leaders (group
// order, fingertip order), over the whole chip — two kernels of CB_GROUPS groups per workgroup (round 4 ran
// one workgroup, which a co-running kernel could starve: 77 µs in the closure against 17 µs alone):
//   screen_count_kernel  sums the select blocks' z-bin histograms, takes the audit cut (cdx_screen.h
//                        audit_bin: the lowest bins within the row budget A, plus the bin that crosses A while
//                        the total stays ≤ 4A — every workgroup computes the same cut), marks each group's
//                        listed rows (kept | audited, keep mask: low byte kept, high byte audited) and writes its
//                        block's counts (listed, audited, discarded) and smallest unaudited z;
//   screen_place_kernel  positions in group order: the listed rows of the earlier blocks (a sum over the
//                        block counts), then a workgroup prefix sum — the same positions as one sequential pass;
//                        block 0 writes the per-closure statistics and the cumulative block.
// Audited beyond the cut: an input-keyed sample of ~1/SAMPLE of the other discarded rows (hash of the row and its
// z), so the audit's checks also reach rows far below the keep threshold.
constexpr int CB_GROUPS = cdx::SCREEN_CB_GROUPS;  // (screen_compact_words sizes the block counts from it)
constexpr unsigned AUDIT_SAMPLE_SHIFT = 9;  // 1 in 512
__device__ __forceinline__ bool audit_sampled(int64_t q, unsigned z) {
  unsigned h = (unsigned)q * 0x9E3779B1u ^ z;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return (h >> (32 - AUDIT_SAMPLE_SHIFT)) == 0u;
}

__device__ __forceinline__ int block_sum(int v, int* red) {  // 256 threads, `red` 4 ints of LDS
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(CB_GROUPS) void screen_count_kernel(int64_t G, int T, int nsel, const int* __restrict__ hist,
                                                                 unsigned short* __restrict__ keep,
                                                                 const unsigned* __restrict__ zkey, int* __restrict__ bcount,
                                                                 int A) {
  __shared__ int s_hist[cdx::AUDIT_BINS];
  __shared__ int red[4], s_cut;
  __shared__ unsigned s_zmin[4];
  const int t = threadIdx.x, lane = t & 63;
  if (A > 0) {  // (eight independent loads in flight per step: the sum is latency-bound, not bandwidth-bound)
    int v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int b = 0;
    for (; b + 8 <= nsel; b += 8)
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] += hist[(int64_t)(b + u) * cdx::AUDIT_BINS + t];
    for (; b < nsel; ++b) v[0] += hist[(int64_t)b * cdx::AUDIT_BINS + t];
    s_hist[t] = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
  }
  if (t == 0) s_cut = A > 0 ? cdx::AUDIT_BINS : 0;
  __syncthreads();
  if (A > 0 && t < 64) {  // the cut: lane l scans bins 4l .. 4l + 3
    constexpr int PB = cdx::AUDIT_BINS / 64;
    int h[PB], sm = 0;
#pragma unroll
    for (int i = 0; i < PB; ++i) sm += (h[i] = s_hist[PB * lane + i]);
    int inc = sm;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(inc, d);
      if (lane >= d) inc += v;
    }
    int c = inc - sm;  // rows in the bins below this lane's
    if (c < A && inc >= A) {  // the lane holding the first bin whose cumulative count reaches A
      int b = 0;
      while (c + h[b] < A) c += h[b++];
      s_cut = PB * lane + b + (c + h[b] <= 4 * A ? 1 : 0);
    }
  }
  __syncthreads();
  const int cut = s_cut;
  const unsigned tmask = (1u << T) - 1u;
  const int64_t gi = (int64_t)blockIdx.x * CB_GROUPS + t;
  int n = 0, na = 0, nd = 0;
  unsigned zmin = 0x7F800000u;  // +inf
  if (gi < G) {
    unsigned m = keep[gi];
    for (int f = 0; f < T; ++f) {
      const int64_t q = gi * T + f;
      const unsigned z = zkey[q];
      if (z == cdx::Z_NONE) continue;
      ++nd;
      if (A > 0 && (cdx::audit_bin(z) < cut || audit_sampled(q, z))) m |= 0x100u << f;
      else zmin = min(zmin, z);
    }
    keep[gi] = (unsigned short)m;
    n = __popc((m | (m >> 8)) & tmask);
    na = __popc(m >> 8);
  }
  n = block_sum(n, red);
  na = block_sum(na, red);
  nd = block_sum(nd, red);
  for (int d = 32; d >= 1; d >>= 1) zmin = min(zmin, (unsigned)__shfl_xor((int)zmin, d));
  if (lane == 0) s_zmin[t >> 6] = zmin;
  __syncthreads();
  if (t == 0) {
    int* o = bcount + 4 * (int64_t)blockIdx.x;
    o[0] = n;
    o[1] = na;
    o[2] = nd;
    o[3] = (int)min(min(s_zmin[0], s_zmin[1]), min(s_zmin[2], s_zmin[3]));
    if (blockIdx.x == 0) bcount[4 * (int64_t)gridDim.x] = cut;
  }
}

__global__ __launch_bounds__(CB_GROUPS) void screen_place_kernel(int64_t G, int T, const unsigned short* __restrict__ keep,
                                                                 const int* __restrict__ bcount, int* __restrict__ vpos,
                                                                 int* __restrict__ rows, int* __restrict__ stats) {
  __shared__ int red[4], wsum[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nb = (int)gridDim.x, b = (int)blockIdx.x;
  // listed rows of the earlier blocks (and, for block 0's statistics, the totals)
  int before = 0;
  for (int i = t; i < b; i += CB_GROUPS) before += bcount[4 * (int64_t)i];
  before = block_sum(before, red);
  const unsigned tmask = (1u << T) - 1u;
  const int64_t gi = (int64_t)b * CB_GROUPS + t;
  const unsigned m = gi < G ? keep[gi] : 0u;
  const int c = __popc((m | (m >> 8)) & tmask);
  int inc = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(inc, d);
    if (lane >= d) inc += v;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  int pos = (int)G + before + inc - c;
  for (int w = 0; w < wave; ++w) pos += wsum[w];
  if (gi < G)
    for (int f = 0; f < T; ++f)
      if (((m >> f) | (m >> (8 + f))) & 1u) {
        const int64_t q = gi * T + f;
        vpos[q] = pos;
        rows[pos] = (int)q;
        ++pos;
      }
  if (b != 0) return;
  int total = 0, total_a = 0, total_d = 0;
  unsigned zm = 0x7F800000u;
  for (int i = t; i < nb; i += CB_GROUPS) {
    const int* o = bcount + 4 * (int64_t)i;
    total += o[0];
    total_a += o[1];
    total_d += o[2];
    zm = min(zm, (unsigned)o[3]);
  }
  total = block_sum(total, red);
  total_a = block_sum(total_a, red);
  total_d = block_sum(total_d, red);
  for (int d = 32; d >= 1; d >>= 1) zm = min(zm, (unsigned)__shfl_xor((int)zm, d));
  __syncthreads();
  if (lane == 0) wsum[wave] = (int)zm;
  __syncthreads();
  if (t == 0) {
    zm = min(min((unsigned)wsum[0], (unsigned)wsum[1]), min((unsigned)wsum[2], (unsigned)wsum[3]));
    stats[cdx::SS_EXTRA] = total;
    stats[cdx::SS_AUDIT] = total_a;
    stats[cdx::SS_GAP] = (int)zm;
    stats[cdx::SS_AUDIT_CUT] = (int)cdx::audit_bin_floor(bcount[4 * (int64_t)nb]);
    stats[cdx::SS_DISCARD] = total_d;
    for (int k : {cdx::SS_MISS, cdx::SS_AUDIT_MISS, cdx::SS_AUDIT_FLIP, cdx::SS_FAULT, cdx::SS_RATIO,
                  cdx::SS_RATIO_AUDIT, cdx::SS_REPAIR})
      stats[k] = 0;
    stats[cdx::SS_CUM] += 1;
    stats[cdx::SS_CUM + cdx::SS_AUDIT] += total_a;
    stats[cdx::SS_CUM + cdx::SS_DISCARD] += total_d;
    unsigned* cz = reinterpret_cast<unsigned*>(stats + cdx::SS_CUM + cdx::SS_GAP);
    *cz = max(*cz, 0xFFFFFFFFu - zm);
  }
}

// Exact values of the kept and audited fingertips from the refine pass's stripe partials, then the
// group's first maximum of log(100·std) — the level kernel's choice — as the ∇std row: sel = its
// query, Xg = its point, vrow = its V row (list position).  Checks every refined row's estimate
// against its margin Δ_f.  A maximum on a row the exact pass did not run (only possible when a
// margin failed) is a fault: the group falls back to its best refined row and its unrefined rows get
// std 0, so the level kernel's argmax agrees and no V row outside the list is read.
// One thread per ROW (round 4; round 3 ran one thread per group, 4 dependent partial-load chains in
// sequence on 64 waves): a workgroup of 64·T threads holds 64 whole groups, each row's exact value,
// check and log(100·std) go through LDS to the group's first thread, which takes the maximum in
// fingertip order.  Counts and maxima are wave-reduced, then one atomic per statistic per wave.
template <int KT>
__global__ __launch_bounds__(64 * CDX_MAX_TIPS) void refine_select_kernel(
    cdx_gpis g, const double* __restrict__ rpartial, int64_t M_pad, int Nt, int64_t G, int T,
    const double* __restrict__ sv2, const int* __restrict__ vpos, const unsigned short* __restrict__ keep,
    const double* __restrict__ X, double* __restrict__ std_, double* __restrict__ var, int64_t* __restrict__ sel,
    double* __restrict__ Xg, int64_t* __restrict__ vrow, int* __restrict__ stats) {
  __shared__ double s_lv[64 * CDX_MAX_TIPS];
  __shared__ int s_pos[64 * CDX_MAX_TIPS];
  const int t = threadIdx.x;
  const int64_t q = (int64_t)blockIdx.x * 64 * T + t;  // this thread's row
  const int64_t gi = q / T;
  const int f = (int)(q - gi * T);
  const bool row = t < 64 * T && gi < G;
  int miss = 0, amiss = 0, aflip = 0, fault = 0;
  float rk = 0.f, ra = 0.f;
  if (row) {
    const double k0 = cdx::gpis_k0<KT>(g.R);
    const int pos = vpos[q];
    double sd;
    if (pos >= 0) {
      double acc = 0;
      for (int s2 = 0; s2 < Nt; ++s2) acc += rpartial[(int64_t)s2 * M_pad + pos];
      const double v = k0 - acc;
      sd = sqrt(fabs(v));
      std_[q] = sd;
      var[q] = v;
      const double* ctr = cdx::screen_view(g).center;
      const double e = fabs(sv2[q] - v),
                   dd = screen_margin(g.screen_delta, ctr, cdx::screen_band(ctr, X[3 * q], X[3 * q + 1], X[3 * q + 2]),
                                      k0, sv2[q]);
      if (isfinite(v) && isfinite(sv2[q])) {
        const float r = (float)(e / dd);
        const bool bad = !(e <= dd);
        if ((keep[gi] >> (8 + f)) & 1u) {
          ra = r;
          amiss = bad;
        } else {
          rk = r;
          miss = bad;
        }
      }
    } else {
      sd = std_[q];
    }
    s_lv[t] = log(100 * sd);
    s_pos[t] = pos;
  }
  __syncthreads();
  if (row && f == 0) {  // the group's first thread: first maximum in fingertip order
    const int t0 = t;
    int fmax = 0, fref = -1;
    double lmax = 0, lref = 0;
    for (int ff = 0; ff < T; ++ff) {
      const double lv = s_lv[t0 + ff];
      const int pos = s_pos[t0 + ff];
      if (ff == 0 || lv > lmax) { lmax = lv; fmax = ff; }
      if (pos >= 0 && (fref < 0 || lv > lref)) { lref = lv; fref = ff; }
    }
    if (s_pos[t0 + fmax] < 0) {
      fault = 1;
      fmax = fref;  // the leader is always refined: fref ≥ 0
      for (int ff = 0; ff < T; ++ff)
        if (s_pos[t0 + ff] < 0) std_[gi * T + ff] = 0.0;
    } else if ((keep[gi] >> (8 + fmax)) & 1u) {
      aflip = 1;  // the exact maximum is an audited row: the screen had discarded it
    }
    const int64_t qi = gi * T + fmax;
    sel[gi] = qi;
    vrow[gi] = s_pos[t0 + fmax];
    for (int i = 0; i < 3; ++i) Xg[3 * gi + i] = X[3 * qi + i];
  }
#pragma unroll
  for (int w = 1; w < 64; w <<= 1) {
    miss += __shfl_xor(miss, w);
    amiss += __shfl_xor(amiss, w);
    aflip += __shfl_xor(aflip, w);
    fault += __shfl_xor(fault, w);
    rk = fmaxf(rk, __shfl_xor(rk, w));
    ra = fmaxf(ra, __shfl_xor(ra, w));
  }
  if ((t & 63) == 0) {
    const int cnt[4] = {miss, amiss, aflip, fault};
    const int idx[4] = {cdx::SS_MISS, cdx::SS_AUDIT_MISS, cdx::SS_AUDIT_FLIP, cdx::SS_FAULT};
    for (int k = 0; k < 4; ++k)
      if (cnt[k]) {
        atomicAdd(&stats[idx[k]], cnt[k]);
        atomicAdd(&stats[cdx::SS_CUM + idx[k]], cnt[k]);
      }
    // non-negative floats order like their bit patterns
    unsigned* us = reinterpret_cast<unsigned*>(stats);
    if (rk > 0.f) {
      atomicMax(&us[cdx::SS_RATIO], __float_as_uint(rk));
      atomicMax(&us[cdx::SS_CUM + cdx::SS_RATIO], __float_as_uint(rk));
    }
    if (ra > 0.f) {
      atomicMax(&us[cdx::SS_RATIO_AUDIT], __float_as_uint(ra));
      atomicMax(&us[cdx::SS_CUM + cdx::SS_RATIO_AUDIT], __float_as_uint(ra));
    }
  }
}

// ------------------------------------------------------------------ preparation (once per state)
// Centre of the inducing points (mean of rows < N, one block, fixed-order tree reduction), the
// centred fp32 copy X1f [N_pad] (padding rows = row 0), the A scale SA and rq² = (max(0, r_safe −
// max_n |x_n − centre|))²: within rq of the centre every |x − x_n| ≤ r_safe, where |SA·Ã| < 2¹⁶.
__global__ __launch_bounds__(256) void screen_center_kernel(cdx_gpis g, double SA, double r_safe, double* __restrict__ center,
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
  __syncthreads();
  double rm = 0;
  for (int j = t; j < g.N; j += 256) {
    const double dx = g.X1[3 * j] - cx, dy = g.X1[3 * j + 1] - cy, dz = g.X1[3 * j + 2] - cz;
    rm = fmax(rm, dx * dx + dy * dy + dz * dz);
  }
  red[0][t] = rm;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[0][t] = fmax(red[0][t], red[0][t + w]);
    __syncthreads();
  }
  if (t == 0) {
    const double rq = fmax(0.0, r_safe - sqrt(red[0][0]));
    center[0] = cx; center[1] = cy; center[2] = cz; center[3] = SA;
    center[4] = isinf(r_safe) ? r_safe : rq * rq;
    center[5] = red[0][0] > 0 ? 4.0 / sqrt(red[0][0]) : 0.0;
    center[6] = center[7] = 0.0;
    for (int b = 0; b < CDX_SCREEN_BANDS; ++b) center[cdx::SCREEN_BAND_OFF + b] = 1.0;
  }
  for (int j = t; j < g.N_pad; j += 256) {
    const int src = j < g.N ? j : 0;
    X1f[j] = make_float4((float)(g.X1[3 * src] - cx), (float)(g.X1[3 * src + 1] - cy), (float)(g.X1[3 * src + 2] - cz),
                         0.f);
  }
}

// L [N_pad/16][2][2][N_pad][8] f16: slice s of SB_j·L⁻ᵀ[16kb + 8h + e][j − shift] (zero for
// j < shift), the B-operand image the screen stages with one 16-byte load per (slice, k-half,
// column).  SB_j = 1/(SA·cscale[j]) (exact powers of two).
__global__ __launch_bounds__(256) void screen_split_kernel(cdx_gpis g, f16x8* __restrict__ L, const double* __restrict__ cscale,
                                                           const double* __restrict__ center) {
  const int Np = g.N_pad, shift = cdx::screen_shift(g.N, Np);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)(Np / 16) * 2 * Np) return;
  const int col = (int)(t % Np);
  const int h = (int)((t / Np) % 2);
  const int kb = (int)(t / (2 * (int64_t)Np));
  const double SB = 1.0 / (cscale[col] * center[3]);
  f16x8 o[2];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int n = 16 * kb + 8 * h + e, j = col - shift;
    const float x = (float)(j >= 0 ? g.Linv_t[(int64_t)n * Np + j] * SB : 0.0);
    const _Float16 a = (_Float16)x;  // round to nearest; x − a is exact in fp32
    o[0][e] = a;
    o[1][e] = (_Float16)(x - (float)a);
  }
  for (int s = 0; s < 2; ++s) L[(((int64_t)kb * 2 + s) * 2 + h) * Np + col] = o[s];
}

// csum[j] = k0 · Σ_{n<N} L⁻ᵀ[n][j − shift] (zero for j < shift): Ṽ = Ã·L⁻ᵀ + csum, and the column's
// product scale cscale[j] = 1/(SA·SB_j) with SB_j = 2^(14 − e), max_n |L⁻ᵀ[n][j − shift]| < 2^e.
// One 1024-thread block per 64 columns: 16 row groups each take every 16th row, then a
// fixed-order combine.
template <int KT>
__global__ __launch_bounds__(1024) void screen_csum_kernel(cdx_gpis g, double SA, double* __restrict__ csum,
                                                           double* __restrict__ cscale) {
  __shared__ double part[16][64], pmax[16][64];
  const int Np = g.N_pad, shift = cdx::screen_shift(g.N, Np);
  const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c, j = col - shift;
  double s = 0, mx = 0;
  if (j >= 0)
    for (int n = rg; n < g.N; n += 16) {
      const double v = g.Linv_t[(int64_t)n * Np + j];
      s += v;
      mx = fmax(mx, fabs(v));
    }
  part[rg][c] = s;
  pmax[rg][c] = mx;
  __syncthreads();
  if (rg == 0) {
    double t = 0;
    for (int r = 0; r < 16; ++r) {
      t += part[r][c];
      mx = fmax(mx, pmax[r][c]);
    }
    csum[col] = cdx::gpis_k0<KT>(g.R) * t;
    int e = 14;
    if (mx > 0) frexp(mx, &e);  // mx < 2^e
    cscale[col] = ldexp(1.0 / SA, e - 14);
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

int screen_audit_rows() {
  static const int n = [] {
    const char* e = cdx::ab_env("CDX_SCREEN_AUDIT");
    return e ? std::max(0, atoi(e)) : 64;
  }();
  return n;
}

int screen_select_launch(const cdx_gpis& g, const double* X, int64_t G, int T, void* ws, double* sv2, double* std_,
                         int* vpos, int* rows, unsigned short* keep, unsigned* zkey, int* stats, hipStream_t s,
                         int (*after_screen)(void*), void* ctx) {
  const int64_t Ms = G * T;
  if (G <= 0 || T <= 0 || T > CDX_MAX_TIPS) return CDX_EINVAL;
  const int64_t M_pad = round_up(Ms, SC_BM);
  const int Nt = g.N_pad / SC_BN;
  if (M_pad / SC_BM * Nt > 0x7fffffff || Ms > 0x7fffffff) return CDX_EINVAL;
  const int Mt = (int)(M_pad / SC_BM);
  double* partial = static_cast<double*>(ws);
  const dim3 grid((unsigned)(Mt * Nt)), sgrid((unsigned)((G + SEL_BLOCK - 1) / SEL_BLOCK));
  const int nsel = (int)sgrid.x, ncb = (int)((G + CB_GROUPS - 1) / CB_GROUPS);
  int* hist = reinterpret_cast<int*>(zkey + G * T);  // screen_compact_words(G) words behind zkey
  int* bcount = hist + (int64_t)nsel * cdx::AUDIT_BINS;
  switch (g.kernel) {
    case CDX_KERNEL_TPS:
      prof_mark(PROF_SCREEN, true, s);
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_TPS>, grid, dim3(SC_THREADS), 0, s, g, X, Ms, partial, M_pad, Mt, Nt);
      prof_mark(PROF_SCREEN, false, s);
      if (after_screen) {
        if (const int r = after_screen(ctx)) return r;
      }
      hipLaunchKernelGGL(screen_select_kernel<CDX_KERNEL_TPS>, sgrid, dim3(SEL_BLOCK), 0, s, g, partial, M_pad, Nt, G, T, sv2, std_, vpos, rows, keep, zkey, X, hist);
      break;
    case CDX_KERNEL_RBF:
      prof_mark(PROF_SCREEN, true, s);
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_RBF>, grid, dim3(SC_THREADS), 0, s, g, X, Ms, partial, M_pad, Mt, Nt);
      prof_mark(PROF_SCREEN, false, s);
      if (after_screen) {
        if (const int r = after_screen(ctx)) return r;
      }
      hipLaunchKernelGGL(screen_select_kernel<CDX_KERNEL_RBF>, sgrid, dim3(SEL_BLOCK), 0, s, g, partial, M_pad, Nt, G, T, sv2, std_, vpos, rows, keep, zkey, X, hist);
      break;
    default:
      prof_mark(PROF_SCREEN, true, s);
      hipLaunchKernelGGL(gpis_screen_kernel<CDX_KERNEL_JOINT>, grid, dim3(SC_THREADS), 0, s, g, X, Ms, partial, M_pad, Mt, Nt);
      prof_mark(PROF_SCREEN, false, s);
      if (after_screen) {
        if (const int r = after_screen(ctx)) return r;
      }
      hipLaunchKernelGGL(screen_select_kernel<CDX_KERNEL_JOINT>, sgrid, dim3(SEL_BLOCK), 0, s, g, partial, M_pad, Nt, G, T, sv2, std_, vpos, rows, keep, zkey, X, hist);
      break;
  }
  hipLaunchKernelGGL(screen_count_kernel, dim3((unsigned)ncb), dim3(CB_GROUPS), 0, s, G, T, nsel, (const int*)hist, keep,
                     (const unsigned*)zkey, bcount, screen_audit_rows());
  hipLaunchKernelGGL(screen_place_kernel, dim3((unsigned)ncb), dim3(CB_GROUPS), 0, s, G, T, (const unsigned short*)keep,
                     (const int*)bcount, vpos, rows, stats);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int refine_select_launch(const cdx_gpis& g, const double* X, int64_t G, int T, const double* rpartial, int64_t M_pad,
                         const double* sv2, const int* vpos, const unsigned short* keep, double* std_, double* var,
                         int64_t* sel, double* Xg, int64_t* vrow, int* stats, hipStream_t s) {
  const int Nt = g.N_pad / SC_BN;
  if (T <= 0 || T > CDX_MAX_TIPS) return CDX_EINVAL;
  const dim3 rgrid((unsigned)((G + 63) / 64));  // 64 groups (64·T rows) per workgroup
  switch (g.kernel) {
    case CDX_KERNEL_TPS:
      hipLaunchKernelGGL(refine_select_kernel<CDX_KERNEL_TPS>, rgrid, dim3(64 * T), 0, s, g, rpartial, M_pad, Nt, G, T, sv2, vpos, keep, X, std_, var, sel, Xg, vrow, stats);
      break;
    case CDX_KERNEL_RBF:
      hipLaunchKernelGGL(refine_select_kernel<CDX_KERNEL_RBF>, rgrid, dim3(64 * T), 0, s, g, rpartial, M_pad, Nt, G, T, sv2, vpos, keep, X, std_, var, sel, Xg, vrow, stats);
      break;
    default:
      hipLaunchKernelGGL(refine_select_kernel<CDX_KERNEL_JOINT>, rgrid, dim3(64 * T), 0, s, g, rpartial, M_pad, Nt, G, T, sv2, vpos, keep, X, std_, var, sel, Xg, vrow, stats);
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
  // SA: k0·SA ∈ (2⁹, 2¹⁰].  r_safe: |Ã(r)| ≤ 49·k0 for r ≤ 3.5R (TPS and the joint kernel's TPS part;
  // R bounds every inducing-point distance), so |SA·Ã| < 2¹⁶ there; the RBF offset is bounded by k0.
  const double k0 = g->kernel == CDX_KERNEL_TPS ? cdx::gpis_k0<CDX_KERNEL_TPS>(g->R)
                    : g->kernel == CDX_KERNEL_RBF ? cdx::gpis_k0<CDX_KERNEL_RBF>(g->R)
                                                  : cdx::gpis_k0<CDX_KERNEL_JOINT>(g->R);
  if (!std::isfinite(k0)) return CDX_EINVAL;
  int ek = 0;
  if (k0 > 0) frexp(k0, &ek);  // k0 < 2^ek (a single inducing point, R = 0: SA = 2¹⁰, rq = 0)
  const double SA = ldexp(1.0, 10 - ek);
  const double r_safe = g->kernel == CDX_KERNEL_RBF ? INFINITY : 3.5 * g->R;
  hipLaunchKernelGGL(screen_center_kernel, dim3(1), dim3(256), 0, s, gv, SA, r_safe, const_cast<double*>(v.center),
                     const_cast<float4*>(v.X1f));
  const dim3 cgrid((unsigned)(Np / 64)), cblk(1024);
  double* csum = const_cast<double*>(v.csum);
  double* cscale = const_cast<double*>(v.cscale);
  switch (g->kernel) {
    case CDX_KERNEL_TPS: hipLaunchKernelGGL(screen_csum_kernel<CDX_KERNEL_TPS>, cgrid, cblk, 0, s, gv, SA, csum, cscale); break;
    case CDX_KERNEL_RBF: hipLaunchKernelGGL(screen_csum_kernel<CDX_KERNEL_RBF>, cgrid, cblk, 0, s, gv, SA, csum, cscale); break;
    default: hipLaunchKernelGGL(screen_csum_kernel<CDX_KERNEL_JOINT>, cgrid, cblk, 0, s, gv, SA, csum, cscale); break;
  }
  const int64_t nsplit = (int64_t)(Np / 16) * 2 * Np;
  hipLaunchKernelGGL(screen_split_kernel, dim3((unsigned)((nsplit + 255) / 256)), dim3(256), 0, s, gv,
                     reinterpret_cast<f16x8*>(const_cast<void*>(v.L)), (const double*)cscale, v.center);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_gpis_screen_info(const cdx_gpis* g, double* out8, cdx_stream_t stream) {
  if (!g || !g->screen || !out8 || g->N_pad <= 0 || g->N_pad % CDX_NPAD_ALIGN) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(out8, cdx::screen_view(*g).center, 8 * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CDX_ELAUNCH;
  return CDX_OK;
}

int cdx_gpis_screen_set_bands(const cdx_gpis* g, const double* w, cdx_stream_t stream) {
  if (!g || !g->screen || !w || g->N_pad <= 0 || g->N_pad % CDX_NPAD_ALIGN) return CDX_EINVAL;
  for (int b = 0; b < CDX_SCREEN_BANDS; ++b)
    if (!(w[b] > 0.0 && w[b] <= 1.0)) return CDX_EINVAL;
  double* dst = const_cast<double*>(cdx::screen_view(*g).center) + cdx::SCREEN_BAND_OFF;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(dst, w, CDX_SCREEN_BANDS * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CDX_ELAUNCH;
  return CDX_OK;
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
