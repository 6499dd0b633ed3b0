// GPIS query kernels for gfx950.
//
//   gpis_mean_kernel   mean = Σ α_j k(x, x_j) + bias and ∇mean (VALU, fp64); optional
//                      normal = ∇mean/(‖∇mean‖+1e-8)   — gpis.py:43-55 (mean), :63-87 (normal)
//   gpis_std_kernel    fp64 MFMA (v_mfma_f64_16x16x4_f64) products with the K* tile generated
//                      on chip, two modes                            — gpis.py:56-59
//                      <VAR>  V = K*·L⁻ᵀ (triangular: N² flops/query), epilogue Σ V²
//                      <!VAR> W = K*·E11⁻¹ (2N² flops/query), epilogue g = Σ_n W kd (x − x_n)
//   gpis_var_finalize  std = sqrt|k0 − ‖L⁻¹k‖²|   (the whitened form: 1e-12 from the reference's
//                      solve, where k·E11⁻¹k with an explicit inverse is 1e-7 on cond 1e7)
//   gpis_grad_finalize ∇std = −sign(v)·g/std, optionally scattered to selected rows
//
// The reference builds the full M×M posterior covariance to read its diagonal and
// re-solves E11 on every call; here E11⁻¹ and α are precomputed once per object and
// only the diagonal is formed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "cdx_gpis.h"
#include "cdx_gpis_launch.h"
#include "cdx_prof.h"
#include "cdx_screen.h"

using cdx::gpis_k;
using cdx::gpis_k0;

typedef double dbl4 __attribute__((ext_vector_type(4)));

namespace {

// Mean kernel: 256-thread workgroups = 16 queries × 16 lanes; each workgroup stages 256
// inducing points (x, y, z, α) per step in LDS and every lane sums a sixteenth of them
// (the 4 lanes of a split read one address), then the 16 lanes of a query reduce with
// xor-shuffles.  The closure's 13·E queries (E = 4096) make 3328 workgroups = 13 waves per SIMD
// over the run: f64-VALU-bound (≈25 f64 ops + one v_rsq_f64 per pair; 0.117 ms for 1.07e8 pairs
// ≈ 90 % of the 30 T f64-op/s the VALU sustains, profiles/r01z_valu_f64.jsonl).  64 × 4 layouts
// (1 wave per SIMD) ran at 0.137 ms; one query per lane with per-wave point ranges (scalar or
// LDS-broadcast reads) at 0.122–0.133 ms (64-query workgroups quantise to 3.25 rounds).
// 32 queries × 8 lanes per workgroup since the moment form (fewer VALU ops per pair, so the
// staging and barriers per pair matter more): 0.095 ms against 0.101 for 16 × 16 and 64 × 4 at
// 53 248 queries (profiles/r02zd_mean_layout_ab.txt).
#ifndef CDX_MEAN_Q  // A/B switches (tools/mean_variants.sh); MEAN_Q · MEAN_SPLIT = 256
#define CDX_MEAN_Q 32
#define CDX_MEAN_SPLIT 8
#endif
constexpr int MEAN_Q = CDX_MEAN_Q, MEAN_SPLIT = CDX_MEAN_SPLIT, MEAN_BLOCK = MEAN_Q * MEAN_SPLIT;
static_assert(MEAN_BLOCK == 256, "the mean kernel's moment reduction assumes 4 waves");

// TPS mean in moment form.  With k = 2r³ − 3Rr² + R³ and ∇k = 6(r − R)(x − x_n):
//   Σ α k   = 2·Σ (αr)·r² − 3R·Σ α r² + R³·Σ α
//   Σ α ∇k  = 6·Σ (αr)(x − x_n) − 6R·Σ α (x − x_n)
// and the r² / (x − x_n) sums are closed forms in the moments S0 = Σ α, S1 = Σ α p̃, S2 = Σ α |p̃|²
// (p̃ = x_n − c, x̃ = x − c, c = the first inducing point, so both stay at the object's scale):
//   Σ α r² = |x̃|² S0 − 2 x̃·S1 + S2,   Σ α (x − x_n) = x̃ S0 − S1.
// Per pair only r, αr, Σ (αr) r² and Σ (αr) d remain: 17 f64 ops + v_rsq against 23 + v_rsq (r
// without the root's final Newton correction, ≤ 1 ulp, as the whitened pass's K* generation).  The product
// build (CDX_MEAN_RSQ32) seeds the root in f32 and takes one f64 Newton step (2⁻⁴⁵ relative, 3 DP ops fewer
// per pair): the mean is DP-issue-bound beside the refine pass, and the closure runs ≈ 10 µs faster (4
// interleaved A/Bs, profiles/r04cde_ab_*.jsonl, r04g_ab_roots.jsonl) while the mean moves by ≤ 6e-13 relative —
// below its own distance from the reference's f64 autograd (1.3e-12 on the banana state, 2.3e-13 on the
// synthetic one; tools/root_precision.py, profiles/r04g_root_precision.jsonl).
// The moments are summed by the staging threads (one point each per block), then over the workgroup.
__device__ __forceinline__ void mean_tps_moments(const cdx_gpis& g, int64_t M, int64_t m, double x0, double x1,
                                                 double x2, double* __restrict__ mean, double* __restrict__ gmean,
                                                 double* __restrict__ normal, dbl4* sp) {
  const int tid = threadIdx.x;
  const int split = tid & (MEAN_SPLIT - 1);
  const double c0 = g.X1[0], c1 = g.X1[1], c2 = g.X1[2];
  double a3 = 0, h0 = 0, h1 = 0, h2 = 0;        // Σ (αr) r², Σ (αr) d
  double s0 = 0, s1x = 0, s1y = 0, s1z = 0, s2 = 0;  // this thread's staged points' moments
  for (int j0 = 0; j0 < g.N; j0 += MEAN_BLOCK) {
    const int j = j0 + tid;
    __syncthreads();
    dbl4 v;
    if (j < g.N) {
      v.x = g.X1[3 * j]; v.y = g.X1[3 * j + 1]; v.z = g.X1[3 * j + 2]; v.w = g.alpha[j];
      const double px = v.x - c0, py = v.y - c1, pz = v.z - c2;
      s0 += v.w;
      s1x += v.w * px; s1y += v.w * py; s1z += v.w * pz;
      s2 += v.w * (px * px + py * py + pz * pz);
    } else {
      v.x = x0 + 1.0; v.y = v.z = 0.0; v.w = 0.0;  // any finite point; α = 0
    }
    sp[tid] = v;
    __syncthreads();
#ifndef CDX_MEAN_UNROLL
#define CDX_MEAN_UNROLL 4
#endif
#pragma unroll CDX_MEAN_UNROLL
    for (int jj = split; jj < MEAN_BLOCK; jj += MEAN_SPLIT) {
      const dbl4 p = sp[jj];
      const double dx = x0 - p.x, dy = x1 - p.y, dz = x2 - p.z;
      const double r2 = dx * dx + dy * dy + dz * dz;
#if defined(CDX_MEAN_RSQ32)  // (product build) f32 seed + one f64 Newton step (≈ 2⁻⁴⁵ relative), see below
      const double ar = p.w * cdx::sqrt_r2_f32seed(r2);
#elif !defined(CDX_MEAN_FULLSQRT)  // the root without its final Newton correction (≤ 1 ulp), as the K* generation
      const double ar = p.w * cdx::sqrt_r2_gen(r2);
#else
      const double ar = p.w * cdx::sqrt_r2(r2);
#endif
      a3 += ar * r2;
      h0 += ar * dx;
      h1 += ar * dy;
      h2 += ar * dz;
    }
  }
#pragma unroll
  for (int w = 1; w < MEAN_SPLIT; w <<= 1) {
    a3 += __shfl_xor(a3, w);
    h0 += __shfl_xor(h0, w);
    h1 += __shfl_xor(h1, w);
    h2 += __shfl_xor(h2, w);
  }
  // workgroup sums of the five moments: wave reduction, then the four waves' partials through LDS
#pragma unroll
  for (int w = 1; w < 64; w <<= 1) {
    s0 += __shfl_xor(s0, w);
    s1x += __shfl_xor(s1x, w);
    s1y += __shfl_xor(s1y, w);
    s1z += __shfl_xor(s1z, w);
    s2 += __shfl_xor(s2, w);
  }
  __syncthreads();
  double* red = reinterpret_cast<double*>(sp);
  const int wave = tid >> 6;
  if ((tid & 63) == 0) {
    red[wave * 5 + 0] = s0; red[wave * 5 + 1] = s1x; red[wave * 5 + 2] = s1y; red[wave * 5 + 3] = s1z;
    red[wave * 5 + 4] = s2;
  }
  __syncthreads();
  s0 = s1x = s1y = s1z = s2 = 0;
#pragma unroll
  for (int w = 0; w < MEAN_BLOCK / 64; ++w) {
    s0 += red[w * 5 + 0]; s1x += red[w * 5 + 1]; s1y += red[w * 5 + 2]; s1z += red[w * 5 + 3];
    s2 += red[w * 5 + 4];
  }
  if (m >= M || split != 0) return;
  const double R = g.R;
  const double qx = x0 - c0, qy = x1 - c1, qz = x2 - c2;
  const double sr2 = (qx * qx + qy * qy + qz * qz) * s0 - 2.0 * (qx * s1x + qy * s1y + qz * s1z) + s2;
  mean[m] = 2.0 * a3 - 3.0 * R * sr2 + R * R * R * s0 + g.bias;
  const double gx = 6.0 * h0 - 6.0 * R * (qx * s0 - s1x);
  const double gy = 6.0 * h1 - 6.0 * R * (qy * s0 - s1y);
  const double gz = 6.0 * h2 - 6.0 * R * (qz * s0 - s1z);
  if (gmean) { gmean[3 * m] = gx; gmean[3 * m + 1] = gy; gmean[3 * m + 2] = gz; }
  if (normal) {
    const double nn = sqrt(gx * gx + gy * gy + gz * gz) + 1e-8;
    normal[3 * m] = gx / nn; normal[3 * m + 1] = gy / nn; normal[3 * m + 2] = gz / nn;
  }
}

// Register-blocked TPS moment form (A/B switch CDX_MEAN_QPT > 1, off): each thread carries MQ_QPT queries, so
// one LDS read of a staged point serves MQ_QPT pairs; MQ_SPLIT lanes share a query group's points.  Same staging,
// moments and epilogue as mean_tps_moments.  Measured slower in the closure (round 5, profiles/r05i_*: the
// mean 85 → 92 µs at 4 queries per thread, 90 µs at 2): the loop is f64-VALU-bound, not LDS-bound, and the
// extra accumulators cost occupancy.
#ifndef CDX_MEAN_QPT
#define CDX_MEAN_QPT 1
#endif
#ifndef CDX_MEAN_QSPLIT
#define CDX_MEAN_QSPLIT 16
#endif
constexpr int MQ_QPT = CDX_MEAN_QPT, MQ_SPLIT = CDX_MEAN_QSPLIT;
constexpr int MQ_PER_WG = (MEAN_BLOCK / MQ_SPLIT) * MQ_QPT;  // queries per workgroup
__global__ __launch_bounds__(MEAN_BLOCK) void gpis_mean_tps_blocked_kernel(cdx_gpis g, const double* __restrict__ X,
                                                                           int64_t M, double* __restrict__ mean,
                                                                           double* __restrict__ gmean,
                                                                           double* __restrict__ normal) {
  __shared__ dbl4 sp[MEAN_BLOCK];
  const int tid = threadIdx.x;
  const int split = tid % MQ_SPLIT;
  const int64_t m0 = ((int64_t)blockIdx.x * (MEAN_BLOCK / MQ_SPLIT) + tid / MQ_SPLIT) * MQ_QPT;
  double xq[MQ_QPT][3];
#pragma unroll
  for (int q = 0; q < MQ_QPT; ++q) {
    const int64_t m = m0 + q;
    for (int i = 0; i < 3; ++i) xq[q][i] = m < M ? X[3 * m + i] : 0.0;
  }
  const double c0 = g.X1[0], c1 = g.X1[1], c2 = g.X1[2];
  double a3[MQ_QPT], h0[MQ_QPT], h1[MQ_QPT], h2[MQ_QPT];
#pragma unroll
  for (int q = 0; q < MQ_QPT; ++q) a3[q] = h0[q] = h1[q] = h2[q] = 0.0;
  double s0 = 0, s1x = 0, s1y = 0, s1z = 0, s2 = 0;
  for (int j0 = 0; j0 < g.N; j0 += MEAN_BLOCK) {
    const int j = j0 + tid;
    __syncthreads();
    dbl4 v;
    if (j < g.N) {
      v.x = g.X1[3 * j]; v.y = g.X1[3 * j + 1]; v.z = g.X1[3 * j + 2]; v.w = g.alpha[j];
      const double px = v.x - c0, py = v.y - c1, pz = v.z - c2;
      s0 += v.w;
      s1x += v.w * px; s1y += v.w * py; s1z += v.w * pz;
      s2 += v.w * (px * px + py * py + pz * pz);
    } else {
      v.x = xq[0][0] + 1.0; v.y = v.z = 0.0; v.w = 0.0;  // any finite point; α = 0
    }
    sp[tid] = v;
    __syncthreads();
#pragma unroll 2
    for (int jj = split; jj < MEAN_BLOCK; jj += MQ_SPLIT) {
      const dbl4 p = sp[jj];
#pragma unroll
      for (int q = 0; q < MQ_QPT; ++q) {
        const double dx = xq[q][0] - p.x, dy = xq[q][1] - p.y, dz = xq[q][2] - p.z;
        const double r2 = dx * dx + dy * dy + dz * dz;
#if defined(CDX_MEAN_RSQ32)
        const double ar = p.w * cdx::sqrt_r2_f32seed(r2);
#else
        const double ar = p.w * cdx::sqrt_r2_gen(r2);
#endif
        a3[q] += ar * r2;
        h0[q] += ar * dx;
        h1[q] += ar * dy;
        h2[q] += ar * dz;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MQ_QPT; ++q)
#pragma unroll
    for (int w = 1; w < MQ_SPLIT; w <<= 1) {
      a3[q] += __shfl_xor(a3[q], w);
      h0[q] += __shfl_xor(h0[q], w);
      h1[q] += __shfl_xor(h1[q], w);
      h2[q] += __shfl_xor(h2[q], w);
    }
#pragma unroll
  for (int w = 1; w < 64; w <<= 1) {
    s0 += __shfl_xor(s0, w);
    s1x += __shfl_xor(s1x, w);
    s1y += __shfl_xor(s1y, w);
    s1z += __shfl_xor(s1z, w);
    s2 += __shfl_xor(s2, w);
  }
  __syncthreads();
  double* red = reinterpret_cast<double*>(sp);
  const int wave = tid >> 6;
  if ((tid & 63) == 0) {
    red[wave * 5 + 0] = s0; red[wave * 5 + 1] = s1x; red[wave * 5 + 2] = s1y; red[wave * 5 + 3] = s1z;
    red[wave * 5 + 4] = s2;
  }
  __syncthreads();
  s0 = s1x = s1y = s1z = s2 = 0;
#pragma unroll
  for (int w = 0; w < MEAN_BLOCK / 64; ++w) {
    s0 += red[w * 5 + 0]; s1x += red[w * 5 + 1]; s1y += red[w * 5 + 2]; s1z += red[w * 5 + 3];
    s2 += red[w * 5 + 4];
  }
  if (split != 0) return;
  const double R = g.R;
#pragma unroll
  for (int q = 0; q < MQ_QPT; ++q) {
    const int64_t m = m0 + q;
    if (m >= M) break;
    const double qx = xq[q][0] - c0, qy = xq[q][1] - c1, qz = xq[q][2] - c2;
    const double sr2 = (qx * qx + qy * qy + qz * qz) * s0 - 2.0 * (qx * s1x + qy * s1y + qz * s1z) + s2;
    mean[m] = 2.0 * a3[q] - 3.0 * R * sr2 + R * R * R * s0 + g.bias;
    const double gx = 6.0 * h0[q] - 6.0 * R * (qx * s0 - s1x);
    const double gy = 6.0 * h1[q] - 6.0 * R * (qy * s0 - s1y);
    const double gz = 6.0 * h2[q] - 6.0 * R * (qz * s0 - s1z);
    if (gmean) { gmean[3 * m] = gx; gmean[3 * m + 1] = gy; gmean[3 * m + 2] = gz; }
    if (normal) {
      const double nn = sqrt(gx * gx + gy * gy + gz * gz) + 1e-8;
      normal[3 * m] = gx / nn; normal[3 * m + 1] = gy / nn; normal[3 * m + 2] = gz / nn;
    }
  }
}

template <int KT>
__global__ __launch_bounds__(MEAN_BLOCK) void gpis_mean_kernel(cdx_gpis g, const double* __restrict__ X, int64_t M,
                                                               double* __restrict__ mean, double* __restrict__ gmean,
                                                               double* __restrict__ normal) {
  __shared__ dbl4 sp[MEAN_BLOCK];  // [point] = (x, y, z, α)
  const int tid = threadIdx.x;
  const int split = tid & (MEAN_SPLIT - 1);
  const int64_t m = (int64_t)blockIdx.x * MEAN_Q + tid / MEAN_SPLIT;
  double x0 = 0, x1 = 0, x2 = 0;
  if (m < M) { x0 = X[3 * m]; x1 = X[3 * m + 1]; x2 = X[3 * m + 2]; }
  const double R = g.R, inv_s2 = 1.0 / (g.sigma * g.sigma);
  double acc = 0, g0 = 0, g1 = 0, g2 = 0;
#ifndef CDX_MEAN_DIRECT  // A/B switch: the per-pair k / ∇k form for TPS too
  if constexpr (KT == CDX_KERNEL_TPS) {
    mean_tps_moments(g, M, m, x0, x1, x2, mean, gmean, normal, sp);
    return;
  }
#endif
  for (int j0 = 0; j0 < g.N; j0 += MEAN_BLOCK) {
    const int j = j0 + tid;
    __syncthreads();
    dbl4 v;
    if (j < g.N) {
      v.x = g.X1[3 * j]; v.y = g.X1[3 * j + 1]; v.z = g.X1[3 * j + 2]; v.w = g.alpha[j];
    } else {
      v.x = x0 + 1.0; v.y = v.z = 0.0; v.w = 0.0;  // any finite point; α = 0
    }
    sp[tid] = v;
    __syncthreads();
#pragma unroll 4
    for (int jj = split; jj < MEAN_BLOCK; jj += MEAN_SPLIT) {
      const dbl4 p = sp[jj];
      const double dx = x0 - p.x, dy = x1 - p.y, dz = x2 - p.z;
      double k, kd;
      gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, k, kd);
      const double a = p.w;
      acc += a * k;
      const double ak = a * kd;
      g0 += ak * dx;
      g1 += ak * dy;
      g2 += ak * dz;
    }
  }
#pragma unroll
  for (int w = 1; w < MEAN_SPLIT; w <<= 1) {
    acc += __shfl_xor(acc, w);
    g0 += __shfl_xor(g0, w);
    g1 += __shfl_xor(g1, w);
    g2 += __shfl_xor(g2, w);
  }
  if (m >= M || split != 0) return;
  mean[m] = acc + g.bias;
  if (gmean) { gmean[3 * m] = g0; gmean[3 * m + 1] = g1; gmean[3 * m + 2] = g2; }
  if (normal) {
    const double nn = sqrt(g0 * g0 + g1 * g1 + g2 * g2) + 1e-8;
    normal[3 * m] = g0 / nn; normal[3 * m + 1] = g1 / nn; normal[3 * m + 2] = g2 / nn;
  }
}

// ------------------------------------------------------------------ std (MFMA)
// 128 queries × 256 output columns per 512-thread workgroup (one per CU: 160 KB of LDS), K-step 16.
// Waves form a 2×4 grid; each owns 64×64 = 4×4 v_mfma_f64_16x16x4_f64 tiles (128 accumulator VGPRs).
// The 256-wide tile halves the per-output-column cost of generating K* on chip against a 128-wide
// tile of 2×2 waves (2.41 vs 2.58 ms at M = 16 384, N = 2000, round-1 A/B).
//
// Three LDS stage buffers: during K-step s the waves multiply out of buffer s%3, stage s+2 is
// generated (K*) / loaded (B) into registers and written to buffer (s+2)%3 after the third substep,
// and the last substep prefetches the first fragments of step s+1 from buffer (s+1)%3 (complete
// since the barrier that ended step s−1).  One barrier per K-step, and nothing waits on LDS right
// after it: the matrix pipe runs across step boundaries (the two-buffer version wrote at the end
// of the step and re-read fragments after the barrier, ≈600 idle pipe cycles per 8192).
// Fragment maps (cdna_hip_programming.md §3, f64 form):
//   A: lane l holds A[row l&15][k l>>4];  B: B[k l>>4][col l&15]
//   C/D: reg r of lane l is D[row (l>>4) + 4r][col l&15]
// K* rows are padded to 144 doubles and B rows to 272 (row stride ≡ 32 dwords mod 64): the two
// half-waves of a ds_read_b64 (rows k, k+1) land on disjoint banks.
constexpr int ST_BM = 128, ST_BK = 16, ST_LD = 144;
constexpr int ST_TILE = ST_BK * ST_LD;                          // doubles per staged K* tile
constexpr int ST_WN = 4;                                        // waves along N
static_assert(CDX_NPAD_ALIGN % (64 * ST_WN) == 0, "N_pad alignment must cover the tile width");
constexpr int ST_BN = 64 * ST_WN;                               // output columns per workgroup
constexpr int ST_THREADS = 128 * ST_WN;                         // 2 row-waves × ST_WN column-waves
constexpr int ST_LDB = ST_BN + 16;                              // padded B row (≡ 32 dwords mod 64)
constexpr int ST_BTILE = ST_BK * ST_LDB;
constexpr int ST_NBUF = 3;                                      // stage buffers
constexpr int ST_XS = 3 * ST_BK;                                // X1 rows of one stage
constexpr int ST_SMEM = ST_NBUF * (ST_TILE + ST_BTILE) + ST_BM * 3 + 2 * ST_XS;
static_assert(ST_SMEM * sizeof(double) <= 160 * 1024, "stage buffers exceed the CU's LDS");

typedef double dbl2v __attribute__((ext_vector_type(2)));

// MODE_GRAD (∇std, explicit inverse): A = K* (generated), B = E11⁻¹, W = K*·E11⁻¹, epilogue
//   Σ W·k and Σ W·kd·(x − x_n) → 4 partials per (column tile, query).
// MODE_VAR (std, whitened): A = K* (generated), B = L⁻ᵀ (upper triangular), V = K*·L⁻ᵀ =
//   (L⁻¹K*ᵀ)ᵀ, epilogue Σ V² → 1 partial per (column tile, query); optionally V itself is stored
//   (vout, [M_pad, N_pad]).  Column tile nt only needs K-rows j < n0 + ST_BN (and < N).
// MODE_GRADV (∇std from the stored whitened vector): A = V rows (loaded, row vsel[m] of vin),
//   B = L⁻¹ (lower triangular), W = V·L⁻¹ = (L⁻ᵀv)ᵀ = (E11⁻¹k)ᵀ, the MODE_GRAD epilogue (linear
//   in W, so K can be split).  Column tile nt only needs K-rows i ≥ n0: N² flops per query
//   instead of 2N²; launched as equal pieces of each query tile's K-sequence (below).
// The triangular modes' tile costs run 1..Nt K-sweeps: stripes are paired heavy+light per XCD.
// (A v_mfma_f64_4x4x4_4b_f64 variant ran no faster — LDS-read-bound, profiles/r01_std_gemm_variants.md.)
// MODE_VARL (the closure's refine pass behind the split-precision screen): MODE_VAR over a device-
//   side row list (rows rl.rows[0 .. G + *rl.extra) of X; V row / partial row = list position),
//   cut into gridDim.x equal pieces of the concatenated K-sequence of all (query tile, stripe)
//   pairs: a piece's segments that cover a whole stripe finish their epilogue in place, a stripe
//   cut by piece boundaries leaves partial V tiles in rl.slots (slot 0: the piece's first segment,
//   1: its last) that gpis_var_merge sums in piece order.  (CDX_MERGE_FUSED instead lets the last of a
//   unit's pieces to finish — a per-unit arrival counter — sum them, in the same order: bit-identical,
//   but 1.22 vs 1.11 ms per closure, profiles/r03f_merge_fused_ab.jsonl: the agent-scope release
//   fence each cut piece needs writes back its XCD's whole L2.)
enum { MODE_GRAD = 0, MODE_VAR = 1, MODE_GRADV = 2, MODE_VARL = 3 };

// Streaming V (A/B switches): CDX_NT_VSTORE stores V rows and the refine's partial tiles non-temporally,
// CDX_NT_VLOAD loads the ∇std pass's V rows non-temporally — streamed once, they then do not evict the
// L⁻ᵀ / L⁻¹ stripes each XCD's L2 re-reads for every query tile.
template <class T>
__device__ __forceinline__ void v_store(T* p, T v) {
#if defined(CDX_NT_VSTORE)
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
// A wave's 64×64 sub-tile of V (acc[i][j][r] = D[row (l>>4) + 4r][col (l&15) + 16j] in block (i, j)) to
// row-major dst (leading dimension ld, even column offset): with CDX_VSTORE_X4 the lane pairs (l, l^1)
// trade one value per two rows (two xor-1 shuffles) so each stores two adjacent columns of two rows as
// 16-byte stores — half the store instructions of the plain 8-byte-per-lane form, same bytes and values.
template <class ACC>
__device__ __forceinline__ void store_v_tile(double* dst, int64_t ld, const ACC& acc, int lane) {
#if defined(CDX_VSTORE_X4)
  const bool even = (lane & 1) == 0;
  const int c0 = (lane & 15) & ~1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double a0 = acc[i][j][0], a1 = acc[i][j][1], a2 = acc[i][j][2], a3 = acc[i][j][3];
      const double x0 = __shfl_xor(even ? a1 : a0, 1), x1 = __shfl_xor(even ? a3 : a2, 1);
      // even lane: rows r = 0, 2 (own value, partner's); odd lane: rows r = 1, 3 (partner's, own value)
      const int ra = even ? 0 : 1, rb = even ? 2 : 3;
      const double2 va = even ? make_double2(a0, x0) : make_double2(x0, a1);
      const double2 vb = even ? make_double2(a2, x1) : make_double2(x1, a3);
      double* base = dst + (int64_t)(16 * i + (lane >> 4)) * ld + 16 * j + c0;
      v_store(reinterpret_cast<double2*>(base + (int64_t)(4 * ra) * ld), va);
      v_store(reinterpret_cast<double2*>(base + (int64_t)(4 * rb) * ld), vb);
    }
#else
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double* vr = dst + (int64_t)(16 * i + (lane >> 4) + 4 * r) * ld + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) v_store(vr + 16 * j, acc[i][j][r]);
    }
#endif
}

template <class T>
__device__ __forceinline__ T v_load(const T* p) {
#if defined(CDX_NT_VLOAD)
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

constexpr int RC_MAX_NT = 16;  // stripes with host unit costs (N_pad ≤ 4096); beyond: equal K-step cuts
static_assert(RC_MAX_NT == cdx::GC_MAX_NT, "the ∇std pass's stripe costs travel in RefineList::uc");
struct RefineList {
  const int* rows;    // query index per list position (null: the identity)
  const int* extra;   // device count of positions past the G primary ones (nullable: 0)
  int G;
  double* slots;      // [gridDim.x][2][ST_BM][ST_BN] partial V tiles of cut stripes
  int* cnt;           // [Nt][mt_cap] arrival counters of cut units (zero between launches)
  int mt_cap;         // query tiles the list can hold
  int64_t* cuts;      // [gridDim.x + 1] piece bounds in the K-sequence (written by the refine kernel)
  int n_uc;           // stripes with unit costs below (= N_pad/256), 0: equal K-step cuts
  int64_t uc[RC_MAX_NT];  // cost of one (stripe, query tile) unit per stripe (var_unit_cost, host)
  const int* gate;    // nullable: screen statistics; the launch has no rows unless cdx::screen_failed
  cdx::RepairSel rs;  // rs.on: the closure's repair pass (whole units, then the selection, see below)
};

// Rows of a refine launch (device-side count; 0 when gated off).
__device__ inline int64_t refine_rows(const RefineList& rl) {
  if (rl.gate && !cdx::screen_failed(rl.gate)) return 0;
  return (int64_t)rl.G + (rl.extra ? *rl.extra : 0);
}

// Whitened pass A operand: K* generated on chip per stripe (default), or read from a buffer
// gpis_kstar_kernel wrote (CDX_VAR_KLOAD).  On chip, each K* entry is regenerated by every stripe
// that needs its row (Σ_nt K-steps = 4.4× the unique ones at N = 2000) and its ≈ 16 f64 VALU ops
// share the DP pipe with the f64 MFMA.  Measured (profiles/r01zi_var_kload_ab.jsonl): the buffer
// makes the std kernel 3 % faster (1.185 → 1.152 ms) but the closure 3 % slower (2.35 → 2.27 M
// evals/s): the 268 MB K* write plus its re-reads slow the K* kernel, mean and ∇std passes more.
#if defined(CDX_VAR_KLOAD)
constexpr bool VAR_KLOAD = true;
#else
constexpr bool VAR_KLOAD = false;
#endif


// K-range [lo, hi) of stripe nt in the triangular modes.
__device__ __host__ inline void stripe_k_range(int mode, int nt, int N, int& lo, int& hi) {
  lo = mode == MODE_GRADV ? nt * ST_BN : 0;
  hi = mode == MODE_GRADV ? N : min(N, nt * ST_BN + ST_BN);
}

// Column shift of the whitened pass: V column j of the pass is L⁻ᵀ column j − var_shift (columns
// below the shift read as zero), i.e. the N_pad − N padding columns (rounded down to whole 16-column
// blocks) sit in front of stripe 0, the lightest stripe (rows [0, 256 − shift)), instead of at the
// end of the heaviest one (all N rows).  N = 2000: 48 columns, stripe pair costs 144 → 138 K-steps.
// The stored V (vout) uses the shifted columns; the ∇std pass reads them back at k + var_shift.
// Capped below one stripe so stripe 0 keeps ≥ 1 live K-step when a caller pads N_pad by ≥ 256.
__device__ __host__ inline int var_shift(int N, int Np) { return min((Np - N) / ST_BK * ST_BK, ST_BN - ST_BK); }

// K-steps of stripe nt's range in the whitened pass (rows [0, min(N, (nt+1)·ST_BN − shift))).
__device__ __host__ inline int var_ksteps(int nt, int N, int Np) {
  const int hi = min(N, (nt + 1) * ST_BN - var_shift(N, Np));
  return (hi + ST_BK - 1) / ST_BK;
}

// K-steps of stripe nt's range in the ∇std pass (rows [nt·ST_BN, N)).
__device__ __host__ inline int gradv_ksteps(int nt, int N) {
  const int lo = nt * ST_BN;
  return N > lo ? (N - lo + ST_BK - 1) / ST_BK : 0;
}

// Refine pass (MODE_VARL) work sequence: the (stripe, query tile) units of var_ksteps(nt) K-steps,
// stripe-major (all tiles of stripe 0, then stripe 1, …), so that the contiguous 1/8 of it each XCD
// runs touches few stripes of L⁻ᵀ (L2 reuse).  Unit containing position q: stripe nt, tile mt,
// sequence range [S0, S1).
__device__ inline void refine_locate(int64_t q, int MtL, int N, int Np, int& nt, int& mt, int64_t& S0, int64_t& S1) {
  int64_t off = 0;
  nt = 0;
  for (;; ++nt) {
    const int64_t len = (int64_t)MtL * var_ksteps(nt, N, Np);
    if (q < off + len || nt == Np / ST_BN - 1) break;
    off += len;
  }
  const int ks = var_ksteps(nt, N, Np);
  mt = (int)((q - off) / ks);
  S0 = off + (int64_t)mt * ks;
  S1 = S0 + ks;
}

// Pieces of the refine pass: one per block (gridDim.x = 256, one per CU), fewer when the sequence is
// short — at least REFINE_MIN_KSTEPS each, so that a cut unit is never spread over dozens of
// nearly empty pieces whose partial tiles the merge would then sum (config-1-sized problems).
constexpr int REFINE_MIN_KSTEPS = 16;
__device__ inline int refine_pieces(int64_t total, int G) {
  return (int)max((int64_t)1, min((int64_t)G, total / REFINE_MIN_KSTEPS));
}
// Piece run by block b: with all G pieces, 32 consecutive ones per XCD (blocks b, b+8, … share an
// XCD); with fewer, piece b (blocks spread round-robin over the XCDs).
__device__ inline int refine_piece(int b, int G, int pieces) {
  return pieces == G && (G & 7) == 0 ? (b & 7) * (G >> 3) + (b >> 3) : b;
}

// Cost-balanced cuts of the refine sequence.  A K-step's time is not uniform: in the last 16–20 K-steps
// of a unit (the stripe's diagonal block) the waves past their own columns skip their MFMAs, so the
// light stripes' short units are cheaper per K-step.  Measured per piece (CDX_DIAG_WGTIME build,
// tools/refine_pieces.py, profiles/r03v_refine_pieces.json): time ≈ 2.8 µs per K-step + 0.27 µs per
// 16-column MFMA block of the busiest SIMD (8 in a full step); equal K-step cuts left the heavy-stripe
// pieces 366 µs against 295 µs for the light ones (end times 292 … 385 µs).  The cuts balance
// RC_FIX + RC_BLK·blocks per K-step instead (integer costs: the same cuts on every workgroup and in the
// merge); CDX_REFINE_UNIFORM builds the equal-K-step cuts for the A/B.
#if defined(CDX_REFINE_UNIFORM)
constexpr int RC_FIX = 1, RC_BLK = 0;
#else
constexpr int RC_FIX = 21, RC_BLK = 2;
#endif
// MFMA blocks (16 columns × one wave) of the busiest SIMD in K-step s of a stripe-nt unit: wave cwave c
// (columns 64c … 64c+63 of the stripe, shifted by vsh) issues 4 blocks up to its diagonal block, then
// 3, 2, 1, 0 (gpis_std_kernel's VAR step variants); SIMDs hold the column waves (c, 3 − c).
__device__ __host__ inline int var_step_blocks(int nt, int s, int vsh16) {
  int b[4];
  for (int c = 0; c < 4; ++c) {
    const int d = s - (16 * nt + 4 * c - vsh16);
    b[c] = d <= 0 ? 4 : (d >= 4 ? 0 : 4 - d);
  }
  return max(b[0] + b[3], b[1] + b[2]);
}
// Piece p of the refine sequence is [cut(p), cut(p+1)).  The per-stripe unit costs depend on (N, N_pad)
// only: the launcher computes them on the host (RefineList::uc); each refine workgroup computes its own
// two bounds from them and the device-side row count (a few scalar steps), and writes its start to
// RefineList::cuts for the merge kernel.
__device__ __host__ inline int64_t var_unit_cost(int nt, int N, int Np) {
  const int vsh16 = var_shift(N, Np) / ST_BK, ks = var_ksteps(nt, N, Np);
  const int sd = min(ks, max(0, 16 * nt - vsh16 + 1));  // steps before the first one below 8 blocks
  int64_t c = (int64_t)sd * (RC_FIX + 8 * RC_BLK);
  for (int s = sd; s < ks; ++s) c += RC_FIX + RC_BLK * var_step_blocks(nt, s, vsh16);
  return c;
}
// ⌊a / b⌋ for 0 ≤ a < 2⁵³, b > 0 through a double division and an exact integer correction
__device__ inline int64_t floordiv_i64(int64_t a, int64_t b) {
  int64_t q = (int64_t)((double)a / (double)b);
  while (q > 0 && q * b > a) --q;
  while ((q + 1) * b <= a) ++q;
  return q;
}
struct RefineCuts {
  int MtL, N, Np, Nt, pieces, vsh16;
  int64_t total;  // K-steps of the sequence
  // start of piece p: the first K-sequence position x whose preceding cost reaches ctot·p/pieces, from
  // the unit costs uc[nt] (a kernel-argument array, indexed statically) and ctot = Σ MtL·uc[nt]
  // (use_uc false: equal K-step cuts)
  template <class UC>
  __device__ __forceinline__ int64_t cut(int p, const UC& uc, bool use_uc, int64_t ctot) const {
    if (p <= 0) return 0;
    if (p >= pieces) return total;
    if (!use_uc) return total * p / pieces;
    const int64_t target = ctot * p;  // compare cost·pieces against ctot·p (exact integers)
    int64_t acc = 0, pos = 0;
#pragma unroll
    for (int nt = 0; nt < RC_MAX_NT; ++nt) {  // static indices into uc (a kernel argument): no scratch copy
      if (nt >= Nt) break;
      const int ks = var_ksteps(nt, N, Np);
      const int64_t sc = (int64_t)MtL * uc[nt];
      if ((acc + sc) * pieces < target) {
        acc += sc;
        pos += (int64_t)MtL * ks;
        continue;
      }
      const int64_t r = target - acc * pieces;  // > 0, ≤ sc·pieces
      const int64_t mt = floordiv_i64(r - 1, uc[nt] * pieces);
      const int64_t need = r - mt * uc[nt] * pieces;  // cost·pieces still to cover inside unit mt
      const int sd = min(ks, max(0, 16 * nt - vsh16 + 1));
      const int64_t full = (RC_FIX + 8 * RC_BLK) * (int64_t)pieces;
      int64_t st;
      if (need <= (int64_t)sd * full) {
        st = floordiv_i64(need + full - 1, full);
      } else {
        int64_t cum = (int64_t)sd * full;
        st = sd;
        while (st < ks && cum < need) cum += (RC_FIX + RC_BLK * var_step_blocks(nt, (int)st++, vsh16)) * (int64_t)pieces;
      }
      return pos + mt * ks + st;
    }
    return total;
  }
};
__device__ inline RefineCuts refine_cuts(const cdx_gpis& g, int64_t Mrows, int G) {
  RefineCuts rc;
  rc.MtL = (int)((Mrows + ST_BM - 1) / ST_BM);
  rc.N = g.N;
  rc.Np = g.N_pad;
  rc.Nt = g.N_pad / ST_BN;
  rc.vsh16 = var_shift(g.N, g.N_pad) / ST_BK;
  int W = 0;
  for (int t = 0; t < rc.Nt; ++t) W += var_ksteps(t, g.N, g.N_pad);
  rc.total = (int64_t)rc.MtL * W;
  rc.pieces = refine_pieces(rc.total, G);
  return rc;
}
// piece holding K-sequence position x: the largest p with cuts[p] ≤ x
__device__ inline int refine_piece_of(int64_t x, const int64_t* cuts, int pieces) {
  int lo = 0, hi = pieces - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cuts[mid] <= x) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// A cut unit (stripe nt, query tile mt, K-sequence [S0, S1)): V = its pieces' partial tiles summed in
// piece order, stored at the list positions, and Σ V² per row into partial[nt][position] — 8 waves,
// 4 columns per lane, MERGE_RB rows per batch so a batch's loads are in flight together.
constexpr int MERGE_THREADS = 512, MERGE_RB = 8;
__device__ inline void refine_merge_unit(const cdx_gpis& g, const RefineList& rl, int64_t M_pad, double* partial,
                                         double* vout, int nt, int mt, int64_t S0, int64_t S1, int pieces, int tid) {
  const int Np = g.N_pad;
  const int pf = refine_piece_of(S0, rl.cuts, pieces), pl = refine_piece_of(S1 - 1, rl.cuts, pieces);
  auto qof = [&](int pp) { return rl.cuts[pp]; };
  const int lane = tid & 63, wave = tid >> 6;
  constexpr int NW = MERGE_THREADS / 64;
  for (int r0 = wave * MERGE_RB; r0 < ST_BM; r0 += NW * MERGE_RB) {
    double v[MERGE_RB][4] = {};
    for (int pp = pf; pp <= pl; ++pp) {
      // this stripe's segment in piece pp; slot 0 if it is the piece's first segment, else 1
      const int64_t a = max(qof(pp), S0), e = min(qof(pp + 1), S1);
      if (a >= e) continue;
      const int slot = 2 * pp + (a == qof(pp) ? 0 : 1);
      const double* src = rl.slots + ((int64_t)slot * ST_BM + r0) * ST_BN + 4 * lane;
#pragma unroll
      for (int rr = 0; rr < MERGE_RB; ++rr)
#pragma unroll
        for (int c = 0; c < 4; ++c) v[rr][c] += src[rr * ST_BN + c];
    }
    double sq[MERGE_RB];
#pragma unroll
    for (int rr = 0; rr < MERGE_RB; ++rr) {
      double* dst = vout + ((int64_t)mt * ST_BM + r0 + rr) * Np + nt * ST_BN + 4 * lane;
      sq[rr] = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        v_store(dst + c, v[rr][c]);
        sq[rr] = fma(v[rr][c], v[rr][c], sq[rr]);
      }
    }
#pragma unroll
    for (int w = 1; w < 64; w <<= 1)
#pragma unroll
      for (int rr = 0; rr < MERGE_RB; ++rr) sq[rr] += __shfl_xor(sq[rr], w);
    if (lane == 0)
#pragma unroll
      for (int rr = 0; rr < MERGE_RB; ++rr) partial[(int64_t)nt * M_pad + (int64_t)mt * ST_BM + r0 + rr] = sq[rr];
  }
}

#if defined(CDX_DIAG_WGTIME)
// timing-only diagnostic: per-workgroup [start, end] (s_memrealtime, 100 MHz), HW_ID, XCC_ID, stripe,
// K-steps of the whitened pass (read back by cdx_diag_wgtime)
__device__ unsigned long long cdx_wgtime[16384][4];
#endif

// VAR, GRAD: one workgroup per (query tile, stripe), partial slot = stripe.  GRADV: a query tile's
// work is the concatenated K-step sequence of its stripes (Σ_nt gradv_ksteps(nt)); it is cut into
// `parts` equal contiguous pieces, one workgroup each, and a piece runs one segment per stripe it
// touches (epilogue per segment, partial slot p + nt: unique, < parts + Nt; the launch lists the
// written slots on the host and the finalize kernel sums them in that fixed order — deterministic).  Equal pieces keep
// every CU equally busy whatever the query count (the closure's 4096 ∇std queries: 32 tiles ×
// 8 pieces = one workgroup of 69 K-steps per CU).
template <int KT, int MODE>
__global__ __launch_bounds__(ST_THREADS, 2) void gpis_std_kernel(cdx_gpis g, const double* __restrict__ X, int64_t M,
                                                                double* __restrict__ partial, int64_t M_pad, int Mt,
                                                                int Nt, double* __restrict__ vout,
                                                                const double* __restrict__ vin,
                                                                const int64_t* __restrict__ vsel, int parts,
                                                                RefineList rl) {
  constexpr bool LIST = MODE == MODE_VARL;
  constexpr bool VAR = MODE == MODE_VAR || LIST;
  constexpr bool TRI = MODE != MODE_GRAD;
  constexpr bool GEN = MODE == MODE_GRAD || (VAR && !VAR_KLOAD);  // A tile generated on chip (else loaded from vin)
  __shared__ __attribute__((aligned(16))) double smem[ST_SMEM];
  double* xq = smem + ST_NBUF * (ST_TILE + ST_BTILE);
  double* xs = xq + ST_BM * 3;  // [2][ST_XS]: X1 rows of the stage generated next
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t Mrows = LIST ? refine_rows(rl) : M;  // rows of this launch (list: device count)
  if (LIST && Mrows == 0) return;                     // a gated repair pass with nothing to repair
#if defined(CDX_DIAG_WGTIME)
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
  const int b = blockIdx.x;
  const double R = g.R, inv_s2 = 1.0 / (g.sigma * g.sigma);
  const int Np = g.N_pad;
  const int vsh = MODE == MODE_GRAD ? 0 : var_shift(g.N, Np);  // VAR: B column shift; GRADV: V column shift
  const double* __restrict__ Bop = VAR ? g.Linv_t : (MODE == MODE_GRADV ? g.Linv : g.Ainv);
  // K* generation: thread → query row gm, GEN_PER k-columns starting at gk (wave-uniform)
  constexpr int GEN_PER = ST_BM * ST_BK / ST_THREADS;  // 4
  static_assert(GEN_PER == 4, "the substep schedule below spreads 4 generated entries over 3 substeps");
  const int gm = tid & (ST_BM - 1);
  const int gk = __builtin_amdgcn_readfirstlane((tid >> 7) * GEN_PER);
  // B tile: 16 rows × ST_BN columns; thread → row ar, four 2-double pieces at columns ac + i·BSTR.
  // Interleaved pieces keep each ds_write_b128 conflict-free (16 consecutive lanes cover the 64
  // banks once; 8 consecutive doubles per thread made it 4-way conflicted, ≈9 % of the K-step)
  // and each global load a contiguous 16 B × 32 lanes.
  constexpr int A_TPR = ST_BN / 8;                      // threads per row
  constexpr int BSTR = 2 * A_TPR;                       // doubles between a thread's pieces
  const int ar = tid / A_TPR, ac = (tid % A_TPR) * 2;
  // wave → 64×64 sub-tile.  Waves w and w+4 share SIMD w%4 (round-robin wave placement); giving
  // them complementary columns (w, 7−w) lets the triangular modes skip the all-zero K-steps of the
  // diagonal block per wave without idling a SIMD (see skip_mfma below).
  const int cwave = wave < 4 ? wave : 7 - wave;
  const int wr = (wave / ST_WN) * 64, wc = __builtin_amdgcn_readfirstlane(cwave * 64);

  // One (query tile mt, stripe nt, K-rows [kbeg, kend)) product and its epilogue into slot pslot.
  auto tile = [&](int mt, int nt, int kbeg, int kend, int pslot, bool full = true) {
  const int64_t m0 = (int64_t)mt * ST_BM;
  const int n0 = nt * ST_BN;
  double qx, qy, qz;
  const double* vrow = nullptr;  // MODE_GRADV: this thread's row of the stored V
  {
    int64_t m = min(m0 + gm, Mrows - 1);  // pad rows replicate a valid query
    if (LIST && rl.rows) m = rl.rows[m];
    qx = X[3 * m]; qy = X[3 * m + 1]; qz = X[3 * m + 2];
    if (tid < ST_BM) { xq[3 * tid] = qx; xq[3 * tid + 1] = qy; xq[3 * tid + 2] = qz; }
    if (!GEN) vrow = vin + (vsel ? vsel[m] : m) * (int64_t)Np;
  }
  // B rows ≥ N are zero: stop at the last live K-step; L⁻ᵀ (VAR) also stops at the tile's
  // diagonal, L⁻¹ (GRADV) starts there
  const int nK = (kend - kbeg + ST_BK - 1) / ST_BK;
  // first row of stage t, clamped at the last stage (the extra stages land in buffers nobody reads)
  auto stage_row = [&](int t) { return kbeg + (t < nK ? t : nK - 1) * ST_BK; };

  dbl2v av[4];
  double kv[GEN_PER];
  auto load_stage = [&](int kb) {  // B rows (and GRADV's V entries) of the stage at row kb
    const dbl2v* src = reinterpret_cast<const dbl2v*>(Bop + (int64_t)(kb + ar) * Np + n0 + ac - (VAR ? vsh : 0));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#if defined(CDX_DIAG_NOBLOAD)  // timing-only diagnostic build: outputs are wrong
      av[i] = dbl2v{qx + kb, qy + i};
#else
      // VAR: the shifted-in columns of stripe 0 are zero (pieces are whole: the shift is a multiple of 16)
      av[i] = (!VAR || n0 != 0 || ac + i * BSTR >= vsh) ? src[i * (BSTR / 2)] : dbl2v{0.0, 0.0};
#endif
    }
    if (!GEN) {  // GRADV: V at shifted columns; VAR: K* rows
#pragma unroll
      for (int i = 0; i < GEN_PER; ++i) kv[i] = v_load(vrow + kb + gk + i + (VAR ? 0 : vsh));
    }
  };
  auto gen = [&](const double* x1, int i) {  // K* entry (gm, gk + i) from the X1 rows at x1
#if defined(CDX_DIAG_NOGEN)  // timing-only diagnostic build: outputs are wrong
    kv[i] = qx - x1[3 * i];
#else
    const double dx = qx - x1[3 * i], dy = qy - x1[3 * i + 1], dz = qz - x1[3 * i + 2];
    double kd;
    gpis_k<KT, true>(dx * dx + dy * dy + dz * dz, R, inv_s2, kv[i], kd);
#endif
  };
  auto stage_write = [&](int buf) {
    double* Kt = smem + buf * (ST_TILE + ST_BTILE);
    double* As = Kt + ST_TILE;
#pragma unroll
    for (int i = 0; i < GEN_PER; ++i) Kt[(gk + i) * ST_LD + gm] = kv[i];
    dbl2v* dst = reinterpret_cast<dbl2v*>(As + ar * ST_LDB + ac);
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i * (BSTR / 2)] = av[i];
  };

  dbl4 acc[4][4];  // [row block][col block] of 16×16
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0, 0, 0, 0};

  // Prologue: stages 0 and 1 into buffers 0 and 1 (X1 straight from global memory), the X1 rows of
  // stage 2 into xs[0].
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kb = stage_row(t);
    load_stage(kb);
    if (GEN) {
#pragma unroll
      for (int i = 0; i < GEN_PER; ++i) gen(g.X1 + 3 * (kb + gk), i);
    }
    stage_write(t);
  }
  if (GEN && tid < ST_XS / 2)
    reinterpret_cast<dbl2v*>(xs)[tid] = reinterpret_cast<const dbl2v*>(g.X1 + 3 * stage_row(2))[tid];
  __syncthreads();

  double fa[2][4], fb[2][4];  // fragment double buffer (substep parity)
  auto frag = [&](int buf, int kk, double* a, double* bb) {
    const double* Kt = smem + buf * (ST_TILE + ST_BTILE);
    const double* As = Kt + ST_TILE;
    const int kra = (kk + (lane >> 4)) * ST_LD + (lane & 15);
    const int krb = (kk + (lane >> 4)) * ST_LDB + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = Kt[kra + wr + 16 * i]; bb[i] = As[krb + wc + 16 * i]; }
  };
  frag(0, 0, fa[0], fb[0]);
  int cb = 0;  // buffer of step s: s % 3
  // The steps of one K-sweep; this wave's MFMA block range [JLO, JHI) per step (see kstep).
  auto step = [&](int s, auto jlo_s, auto jhi_s) {
    const int nb = cb == ST_NBUF - 1 ? 0 : cb + 1, wb = nb == ST_NBUF - 1 ? 0 : nb + 1;
    load_stage(stage_row(s + 2));
    // X1 rows of stage s+3 (staged through LDS by the first 24 lanes: the generation then issues no
    // scalar loads, whose lgkmcnt waits would also drain the fragment reads in flight)
    dbl2v xl = dbl2v{0, 0};
    if (GEN && tid < ST_XS / 2) xl = reinterpret_cast<const dbl2v*>(g.X1 + 3 * stage_row(s + 3))[tid];
    const double* x1 = xs + (s & 1) * ST_XS + 3 * gk;
    // This wave's B columns (true columns [c0, c0 + 64)) are all zero for the whole K-step when the
    // step lies past their diagonal (L⁻ᵀ, VAR) or before it (L⁻¹, GRADV): skip the MFMAs, keep the
    // staging and barriers.  Inside the diagonal block (K-step t = 0..3 of it) the 16-column blocks
    // j < t (VAR) or j > t (GRADV) are zero too: those variants issue only the live blocks' MFMAs
    // (compile-time block ranges, no per-block predicate).  acc + 0·A is acc: bit-identical.
    auto kstep = [&](auto jlo_c, auto jhi_c) {
      constexpr int JLO = decltype(jlo_c)::value, JHI = decltype(jhi_c)::value;  // live blocks [JLO, JHI)
#pragma unroll
      for (int kk = 0; kk < ST_BK; kk += 4) {
        const int cur = (kk >> 2) & 1;
        // next substep's fragments; the last substep reads step s+1's first ones
        if (kk + 4 < ST_BK) frag(cb, kk + 4, fa[cur ^ 1], fb[cur ^ 1]);
        else frag(nb, 0, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = JLO; j < JHI; ++j) {
#if defined(CDX_DIAG_NOMFMA)  // timing-only diagnostic build: outputs are wrong
            acc[i][j][0] += fa[cur][i] * fb[cur][j];
#else
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0);
#endif
          }
        // stage s+2: K* entries over substeps 0–2 (2, 1, 1), written after substep 2's MFMAs
        if (GEN) {
          if (kk == 0) { gen(x1, 0); gen(x1, 1); }
          if (kk == 4) gen(x1, 2);
          if (kk == 8) gen(x1, 3);
        }
        if (kk == 8) stage_write(wb);
#if defined(CDX_STD_SCHED)
        if constexpr (JHI > JLO) {
          __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // next fragments first
#pragma unroll
          for (int q = 0; q < 4 * (JHI - JLO); ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // then up to four VALU
          }
        }
#endif
      }
    };
    kstep(jlo_s, jhi_s);
    if (GEN && tid < ST_XS / 2) reinterpret_cast<dbl2v*>(xs + ((s + 1) & 1) * ST_XS)[tid] = xl;
    cb = nb;
    __syncthreads();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  // K-step s sits at dt = s + d0 relative to this wave's 64-row diagonal block (true columns
  // [c0, c0 + 64)); the diagonal variants run in their own straight-line calls, so each loop keeps
  // one fragment schedule (a per-step dispatch inside one loop made the allocator spill).
  const int c0 = n0 + wc - (VAR ? vsh : 0);
  const int d0 = (kbeg - c0) >> 4;  // kbeg − c0 is a multiple of 16; wave-uniform
  int s = 0;
  if constexpr (VAR) {
    for (const int e = min(nK, max(0, 1 - d0)); s < e; ++s) step(s, I0{}, I4{});
#if !defined(CDX_STD_NODIAG)
    if (s < nK && s + d0 == 1) step(s++, I1{}, I4{});
    if (s < nK && s + d0 == 2) step(s++, I2{}, I4{});
    if (s < nK && s + d0 == 3) step(s++, I3{}, I4{});
#else
    for (const int e = min(nK, max(0, 4 - d0)); s < e; ++s) step(s, I0{}, I4{});
#endif
    for (; s < nK; ++s) step(s, I0{}, I0{});
  } else if constexpr (MODE == MODE_GRADV) {
    for (const int e = min(nK, max(0, -d0)); s < e; ++s) step(s, I0{}, I0{});
#if !defined(CDX_STD_NODIAG)
    if (s < nK && s + d0 == 0) step(s++, I0{}, I1{});
    if (s < nK && s + d0 == 1) step(s++, I0{}, I2{});
    if (s < nK && s + d0 == 2) step(s++, I0{}, I3{});
#endif
    for (; s < nK; ++s) step(s, I0{}, I4{});
  } else {
    for (; s < nK; ++s) step(s, I0{}, I4{});
  }

  if constexpr (VAR) {
    // Epilogue: per owned row Σ V² over this wave's 64 columns, reduced over the 16 lanes of a
    // row, then over the column waves in LDS; V itself to vout when asked (16 lanes of a row write
    // 128 contiguous bytes).  Split-K launches (parts > 0) store their K-chunk's partial V tile to
    // partial[pslot = chunk][M_pad][N_pad] instead; gpis_var_splitk_finalize sums the chunks.
    double* red = smem;  // [ST_WN][ST_BM]
    if (LIST && !full) {  // a cut stripe: this segment's partial V tile to its slot
#if !defined(CDX_DIAG_NOVSTORE)  // timing-only diagnostic build (outputs wrong): no V / partial-tile stores
      store_v_tile(rl.slots + ((int64_t)pslot * ST_BM + wr) * ST_BN + wc, ST_BN, acc, lane);
#endif
      return;
    }
    if (!LIST && parts > 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double* vr = partial + ((int64_t)pslot * M_pad + m0 + wr + 16 * i + (lane >> 4) + 4 * r) * Np + n0 + wc +
                       (lane & 15);
#pragma unroll
          for (int j = 0; j < 4; ++j) vr[16 * j] = acc[i][j][r];
        }
      return;
    }
#if defined(CDX_DIAG_NOVSTORE)
    if (vout && !LIST) {
#else
    if (vout) {
#endif
      store_v_tile(vout + (m0 + wr) * (int64_t)Np + n0 + wc, Np, acc, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double v = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) v = fma(acc[i][j][r], acc[i][j][r], v);
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if ((lane & 15) == 0) red[cwave * ST_BM + wr + 16 * i + (lane >> 4) + 4 * r] = v;
      }
    }
    __syncthreads();
    if (tid < ST_BM) {
      double v = 0.0;
#pragma unroll
      for (int w = 0; w < ST_WN; ++w) v += red[w * ST_BM + tid];
      partial[(int64_t)pslot * M_pad + m0 + tid] = v;
    }
#if defined(CDX_DIAG_WGTIME)
    if (tid == 0 && b < 16384) {
      cdx_wgtime[b][0] = t_start;
      cdx_wgtime[b][1] = __builtin_amdgcn_s_memrealtime();
      cdx_wgtime[b][2] = ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32) |
                         (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
      cdx_wgtime[b][3] = ((unsigned long long)nt << 32) | (unsigned)nK;
    }
#endif
    return;
  }

  // Epilogue: per owned row g = Σ_n W kd (x_m − x_n) over this wave's 64 columns (slot 0 of the
  // 4-double partial stays 0), reduced over the 16 lanes of a row (xor-shuffles), then over the
  // column waves in LDS.
  double* red = smem;  // [ST_WN][ST_BM][4], reuses the staging buffers (loop ended on a barrier)
  double nxs[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc + 16 * j + (lane & 15);
    nxs[j][0] = g.X1[3 * n]; nxs[j][1] = g.X1[3 * n + 1]; nxs[j][2] = g.X1[3 * n + 2];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double ps[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ps[r][0] = ps[r][1] = ps[r][2] = ps[r][3] = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = wr + 16 * i + (lane >> 4) + 4 * r;
      const double mx = xq[3 * row], my = xq[3 * row + 1], mz = xq[3 * row + 2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double dx = mx - nxs[j][0], dy = my - nxs[j][1], dz = mz - nxs[j][2];
        double k, kd;
        gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, k, kd);
        const double wkd = acc[i][j][r] * kd;
        ps[r][1] += wkd * dx;
        ps[r][2] += wkd * dy;
        ps[r][3] += wkd * dz;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        double v = ps[r][c];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        ps[r][c] = v;
      }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr + 16 * i + (lane >> 4) + 4 * r;
#pragma unroll
        for (int c = 0; c < 4; ++c) red[(cwave * ST_BM + row) * 4 + c] = ps[r][c];
      }
    }
  }
  __syncthreads();
  for (int idx = tid; idx < ST_BM * 4; idx += ST_THREADS) {
    const int row = idx >> 2, c = idx & 3;
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < ST_WN; ++w) v += red[(w * ST_BM + row) * 4 + c];
    partial[((int64_t)pslot * M_pad + m0 + row) * 4 + c] = v;
  }
  };  // tile

  if constexpr (LIST) {
    if (rl.rs.on) {
      // The repair pass (gated: only after a failed check, so its speed does not matter): whole units
      // u = b, b + gridDim.x, … (no cut stripes, no merge), then the last workgroup to finish — an arrival
      // counter in the workspace, released / acquired at agent scope — takes every group's exact
      // selection (the unscreened closure's): std / var of all rows, the first maximum of log(100·std).
      const int MtL = (int)((Mrows + ST_BM - 1) / ST_BM), Ntl = Np / ST_BN;
      bool first_u = true;
      for (int u = b; u < MtL * Ntl; u += gridDim.x) {
        const int nt = u / MtL, mt = u - nt * MtL;
        if (!first_u) __syncthreads();  // the previous unit's epilogue used the stage buffers
        first_u = false;
        tile(mt, nt, 0, min(g.N, nt * ST_BN + ST_BN - vsh), nt, true);
      }
      __shared__ int s_lastwg;
      __threadfence();
      __syncthreads();
      if (tid == 0) {
        s_lastwg = atomicAdd(rl.rs.done, 1) == (int)gridDim.x - 1;
        if (s_lastwg) {
          *rl.rs.done = 0;  // ready for the next launch
          rl.rs.stats[cdx::SS_REPAIR] = 1;  // (not among the words screen_failed reads)
          rl.rs.stats[cdx::SS_CUM + cdx::SS_REPAIR] += 1;
        }
      }
      __syncthreads();
      if (!s_lastwg) return;
      __threadfence();
      const double k0 = gpis_k0<KT>(g.R);
      for (int64_t gi = tid; gi < rl.rs.G; gi += ST_THREADS) {
        int fmax = 0;
        double lmax = 0;
        for (int f = 0; f < rl.rs.T; ++f) {
          const int64_t q = gi * rl.rs.T + f;
          double acc = 0;
          for (int t = 0; t < Ntl; ++t) acc += partial[(int64_t)t * M_pad + q];
          const double v = k0 - acc, sd = sqrt(fabs(v));
          rl.rs.std_[q] = sd;
          rl.rs.var[q] = v;
          const double lv = log(100 * sd);
          if (f == 0 || lv > lmax) { lmax = lv; fmax = f; }
        }
        const int64_t qi = gi * rl.rs.T + fmax;
        rl.rs.sel[gi] = qi;
        rl.rs.vrow[gi] = qi;
        for (int i = 0; i < 3; ++i) rl.rs.Xg[3 * gi + i] = X[3 * qi + i];
      }
      return;
    }
    // pieces of the concatenated K-sequence of all (stripe, query tile) units (refine_locate)
    const RefineCuts rc = refine_cuts(g, Mrows, gridDim.x);
    const int MtL = rc.MtL, pieces = rc.pieces;
    const int pc = refine_piece(b, gridDim.x, pieces);
    if (pc >= pieces) return;
    const bool use_uc = rl.n_uc == rc.Nt && rc.total >= 32 * (int64_t)pieces;  // short pieces: equal K-steps
    int64_t ctot = 0;
#pragma unroll
    for (int nt = 0; nt < RC_MAX_NT; ++nt)
      if (nt < rc.Nt) ctot += (int64_t)MtL * rl.uc[nt];
    const int64_t q0 = rc.cut(pc, rl.uc, use_uc, ctot), q1 = rc.cut(pc + 1, rl.uc, use_uc, ctot);
    if (tid == 0) {  // the piece table for the merge kernel
      rl.cuts[pc] = q0;
      if (pc == pieces - 1) rl.cuts[pieces] = q1;
    }
    bool first = true;
    __shared__ int s_last;
#if defined(CDX_DIAG_WGTIME)
    int n_seg = 0;
#endif
    for (int64_t q = q0; q < q1;) {
      int nt, mt;
      int64_t S0, S1;
      refine_locate(q, MtL, g.N, Np, nt, mt, S0, S1);
      const int64_t e = min(q1, S1);
      const int hi = min(g.N, nt * ST_BN + ST_BN - vsh);
      const int kbeg = (int)(q - S0) * ST_BK, kend = min(hi, (int)(e - S0) * ST_BK);
      const bool full = q == S0 && e == S1;
      if (!first) __syncthreads();  // the previous segment's epilogue used the stage buffers
      first = false;
      tile(mt, nt, kbeg, kend, full ? nt : 2 * pc + (q == q0 ? 0 : 1), full);
#if defined(CDX_MERGE_FUSED)
      if (!full) {
        // release this piece's partial tile, count the arrival; the unit's last piece merges it
        __threadfence();
        __syncthreads();
        if (tid == 0) {
          const int n = refine_piece_of(S1 - 1, rl.cuts, pieces) - refine_piece_of(S0, rl.cuts, pieces) + 1;
          int* c = rl.cnt + (int64_t)nt * rl.mt_cap + mt;
          const int old = atomicAdd(c, 1);
          s_last = old == n - 1;
          if (old == n - 1) *c = 0;  // ready for the next launch
        }
        __syncthreads();
        if (s_last) {
          __threadfence();  // acquire: the other pieces' tiles
          refine_merge_unit(g, rl, M_pad, partial, vout, nt, mt, S0, S1, pieces, tid);
        }
      }
#endif
      q = e;
#if defined(CDX_DIAG_WGTIME)
      ++n_seg;
#endif
    }
#if defined(CDX_DIAG_WGTIME)  // the piece's [start, end], HW ids, (segments, K-steps)
    if (tid == 0 && b < 16384) {
      cdx_wgtime[b][0] = t_start;
      cdx_wgtime[b][1] = __builtin_amdgcn_s_memrealtime();
      cdx_wgtime[b][2] = ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32) |
                         (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
      cdx_wgtime[b][3] = ((unsigned long long)n_seg << 32) | (unsigned)(q1 - q0);
    }
#endif
    return;
  }
  if (MODE == MODE_GRADV) {
    const int U = Mt * parts;
    const int t = (U & 7) == 0 ? (b & 7) * (U >> 3) + (b >> 3) : b;  // each XCD: one K-range, many tiles
    const int p = t / Mt, mt = t - p * Mt;
    int W = 0;
    for (int nt = 0; nt < Nt; ++nt) W += gradv_ksteps(nt, g.N);
    // cost-balanced cuts from the launcher's per-stripe costs (carried in rl.uc, RC_MAX_NT = GC_MAX_NT)
    const int q0 = cdx::gradv_cut(p, parts, W, g.N, Nt, rl.uc, rl.n_uc),
              q1 = cdx::gradv_cut(p + 1, parts, W, g.N, Nt, rl.uc, rl.n_uc);
    bool first = true;
    for (int nt = 0, s0 = 0; nt < Nt; ++nt) {
      const int s1 = s0 + gradv_ksteps(nt, g.N);
      const int a = max(q0, s0), e = min(q1, s1);
      if (a < e) {
        if (!first) __syncthreads();  // the previous segment's epilogue used the stage buffers
        first = false;
        tile(mt, nt, nt * ST_BN + (a - s0) * ST_BK, min(g.N, nt * ST_BN + (e - s0) * ST_BK), p + nt);
      }
      s0 = s1;
    }
    return;
  }
  int nt, mt;
  if (VAR && parts > 0) {
    // Split-K (few query tiles): unit = (stripe nt, K-chunk c of `parts` K-steps, query tile); the
    // units of one (nt, c) block are consecutive, block-major.
    int blk = b / Mt;
    mt = b - blk * Mt;
    for (nt = 0;; ++nt) {
      const int nch = (var_ksteps(nt, g.N, g.N_pad) + parts - 1) / parts;
      if (blk < nch) break;
      blk -= nch;
    }
    const int k0 = blk * parts * ST_BK;
    tile(mt, nt, k0, min(min(g.N, nt * ST_BN + ST_BN - vsh), k0 + parts * ST_BK), blk);
    return;
  }
  if (TRI) {
    // Stripe nt costs ∝ nt + 1 K-sweeps.  Pair stripes (Nt−1−a, a) — every pair costs Nt + 1 — and
    // give each pair to X = 16/Nt XCDs (blocks b, b+8, … share an XCD), each XCD taking 1/X of the
    // pair's query tiles, heavy stripe first: equal work per XCD, and each XCD's L2 holds only its
    // two stripes of L⁻ᵀ (each stripe is fetched by X XCDs instead of all eight).
    const int X = 16 / Nt;
    if (Nt >= 2 && Nt <= 16 && (Nt & (Nt - 1)) == 0 && Mt % X == 0) {
      const int xcd = b & 7, r = b >> 3, per = Mt / X;
      const int a = xcd / X, part = xcd % X;
      nt = r < per ? Nt - 1 - a : a;
      mt = part * per + (r < per ? r : r - per);
    } else {  // heaviest stripe first
      nt = Nt - 1 - b / Mt;
      mt = b % Mt;
    }
  } else {
    // XCD-aware order: blocks b and b+8 share an XCD (round-robin dispatch); give each XCD a
    // contiguous run of n-major tiles so its L2 serves the same E11⁻¹ column stripes.
    const int T = Mt * Nt;
    const int t = (T & 7) == 0 ? (b & 7) * (T >> 3) + (b >> 3) : b;
    nt = t / Mt;
    mt = t - nt * Mt;
  }
  // B rows ≥ N are zero: stop at the last live K-step; L⁻ᵀ (VAR) also stops at the tile's diagonal
  tile(mt, nt, 0, VAR ? min(g.N, nt * ST_BN + ST_BN - vsh) : g.N, nt);
}



// K*[m][j] = k(x_m, x_j) for j < N, 0 for N ≤ j < N_pad: the whitened pass's A operand
// ([M][N_pad], row-major).  Each 256-thread block covers KS_ROWS query rows: a thread keeps one
// inducing point per column step and writes KS_ROWS rows (coalesced along j); X1 is read once
// per block.  Write-bound: 8·N_pad bytes per query.
constexpr int KS_ROWS = 16;
template <int KT>
__global__ __launch_bounds__(256) void gpis_kstar_kernel(cdx_gpis g, const double* __restrict__ X, int64_t M,
                                                         double* __restrict__ out) {
  __shared__ double xq[3 * KS_ROWS];
  const int64_t m0 = (int64_t)blockIdx.x * KS_ROWS;
  const int Np = g.N_pad, N = g.N;
  if (threadIdx.x < 3 * KS_ROWS) {
    const int64_t m = min(m0 + threadIdx.x / 3, M - 1);
    xq[threadIdx.x] = X[3 * m + threadIdx.x % 3];
  }
  __syncthreads();
  const double R = g.R, inv_s2 = 1.0 / (g.sigma * g.sigma);
  const int nr = (int)min((int64_t)KS_ROWS, M - m0);
  for (int j = threadIdx.x; j < Np; j += 256) {
    const bool live = j < N;
    const double px = live ? g.X1[3 * j] : 0.0, py = live ? g.X1[3 * j + 1] : 0.0, pz = live ? g.X1[3 * j + 2] : 0.0;
    for (int r = 0; r < nr; ++r) {
      const double dx = xq[3 * r] - px, dy = xq[3 * r + 1] - py, dz = xq[3 * r + 2] - pz;
      double k, kd;
      gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, k, kd);
      out[(m0 + r) * Np + j] = live ? k : 0.0;
    }
  }
}

// std = sqrt|k0 − Σ_t V²-partials|; var_out keeps the signed k0 − ‖L⁻¹k‖² for the ∇std scale.
template <int KT>
__global__ __launch_bounds__(256) void gpis_var_finalize(cdx_gpis g, const double* __restrict__ partial, int64_t M,
                                                         int64_t M_pad, int n_tiles, double* __restrict__ std_out,
                                                         double* __restrict__ var_out) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  double s = 0;
  for (int t = 0; t < n_tiles; ++t) s += partial[(int64_t)t * M_pad + m];
  const double v = gpis_k0<KT>(g.R) - s;
  std_out[m] = sqrt(fabs(v));
  if (var_out) var_out[m] = v;
}

// argmax over the T rows of group t of log(100·std) (first maximum), as level_fwd_bwd picks it.
__device__ inline void group_select(int64_t t, int T, const double* __restrict__ std_, const double* __restrict__ X,
                                    int64_t* __restrict__ sel, double* __restrict__ Xg) {
  int fmax = 0;
  double lmax = log(100 * std_[t * T]);
  for (int f = 1; f < T; ++f) {
    const double lv = log(100 * std_[t * T + f]);
    if (lv > lmax) { lmax = lv; fmax = f; }
  }
  const int64_t qi = t * T + fmax;
  sel[t] = qi;
  for (int i = 0; i < 3; ++i) Xg[3 * t + i] = X[3 * qi + i];
}

// gpis_var_finalize (one thread per row), then each group's selection by its first row's thread
// from the block's LDS copy of log(100·std) (T divides the 256-row block: groups never straddle).
template <int KT>
__global__ __launch_bounds__(256) void gpis_var_finalize_select(cdx_gpis g, const double* __restrict__ partial,
                                                                int64_t M, int T, int64_t M_pad, int n_tiles,
                                                                double* __restrict__ std_out,
                                                                double* __restrict__ var_out,
                                                                const double* __restrict__ X,
                                                                int64_t* __restrict__ sel, double* __restrict__ Xg) {
  __shared__ double lg[256];
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m < M) {
    double s = 0;
    for (int t = 0; t < n_tiles; ++t) s += partial[(int64_t)t * M_pad + m];
    const double v = gpis_k0<KT>(g.R) - s;
    const double sd = sqrt(fabs(v));
    std_out[m] = sd;
    if (var_out) var_out[m] = v;
    lg[threadIdx.x] = log(100 * sd);
  }
  __syncthreads();
  if (m >= M || m % T != 0) return;
  int fmax = 0;
  double lmax = lg[threadIdx.x];
  for (int f = 1; f < T; ++f) {
    const double lv = lg[threadIdx.x + f];
    if (lv > lmax) { lmax = lv; fmax = f; }
  }
  const int64_t t = m / T, qi = m + fmax;
  sel[t] = qi;
  for (int i = 0; i < 3; ++i) Xg[3 * t + i] = X[3 * qi + i];
}

__global__ __launch_bounds__(256) void gpis_select_kernel(int64_t G, int T, const double* __restrict__ std_,
                                                          const double* __restrict__ X, int64_t* __restrict__ sel,
                                                          double* __restrict__ Xg) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < G) group_select(t, T, std_, X, sel, Xg);
}

// Split-K whitened pass: V[m, col] = Σ_c chunk partials (fixed order), stored to vout when asked,
// std = sqrt|k0 − Σ_col V²| — one 256-thread block per query row, tree-reduced (deterministic).
template <int KT>
__global__ __launch_bounds__(256) void gpis_var_splitk_finalize(cdx_gpis g, const double* __restrict__ vpart,
                                                                int64_t M_pad, int chunk, double* __restrict__ vout,
                                                                double* __restrict__ std_out,
                                                                double* __restrict__ var_out) {
  __shared__ double red[256];
  const int64_t m = blockIdx.x;
  const int Np = g.N_pad;
  double s = 0;
  for (int col = threadIdx.x; col < Np; col += 256) {
    const int nch = (var_ksteps(col / ST_BN, g.N, Np) + chunk - 1) / chunk;
    double v = 0;
    for (int c = 0; c < nch; ++c) v += vpart[((int64_t)c * M_pad + m) * Np + col];
    if (vout) vout[m * Np + col] = v;
    s = fma(v, v, s);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double v = gpis_k0<KT>(g.R) - red[0];
    std_out[m] = sqrt(fabs(v));
    if (var_out) var_out[m] = v;
  }
}

#if !defined(CDX_MERGE_FUSED)
// The cut units merged by a separate kernel after the refine pass — workgroup p finishes the unit
// whose K-range ends inside piece p after starting in an earlier one.
__global__ __launch_bounds__(MERGE_THREADS) void gpis_var_merge(cdx_gpis g, RefineList rl, int64_t M_pad,
                                                      double* __restrict__ partial, double* __restrict__ vout) {
  const int64_t Mrows = refine_rows(rl);
  if (Mrows == 0) return;
  const RefineCuts rc = refine_cuts(g, Mrows, gridDim.x);
  const int p = blockIdx.x;
  if (p >= rc.pieces) return;
  const int64_t q0 = rl.cuts[p], q1 = rl.cuts[p + 1];
  if (q0 >= q1 || q0 >= rc.total) return;
  int nt, mt;
  int64_t S0, S1;
  refine_locate(q0, rc.MtL, g.N, g.N_pad, nt, mt, S0, S1);
  if (!(S0 < q0 && S1 <= q1)) return;
  refine_merge_unit(g, rl, M_pad, partial, vout, nt, mt, S0, S1, rc.pieces, threadIdx.x);
}

#endif

// Partial slots a ∇std launch wrote, in increasing order (host-computed, passed by value).
constexpr int GRAD_MAX_SLOTS = 512;
struct GradSlots {
  int n;
  unsigned short t[GRAD_MAX_SLOTS];
};

// ∇std = −sign(v)·(Σ_n W kd (x − x_n))/sqrt|v| at query m, written to row sel[m] (identity when
// sel is null) with v = var[sel[m]] from the whitened pass.  Sums the listed slots in order: all
// stripes (GRAD), or only the slots p + nt the GRADV pieces wrote (no memset of the others).
__global__ __launch_bounds__(256) void gpis_grad_finalize(const double* __restrict__ partial, int64_t M,
                                                          int64_t M_pad, const GradSlots slots,
                                                          const int64_t* __restrict__ sel,
                                                          const double* __restrict__ var, double* __restrict__ gstd) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  double g0 = 0, g1 = 0, g2 = 0;
  for (int i = 0; i < slots.n; ++i) {
    const double* p = partial + ((int64_t)slots.t[i] * M_pad + m) * 4;
    g0 += p[1]; g1 += p[2]; g2 += p[3];
  }
  const int64_t o = sel ? sel[m] : m;
  const double v = var[o];
  const double sg = v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0);
  const double f = -sg / sqrt(fabs(v));
  gstd[3 * o] = f * g0; gstd[3 * o + 1] = f * g1; gstd[3 * o + 2] = f * g2;
}

__global__ void mfma_f64_selftest_kernel(const double* A, const double* B, double* D) {
  const int lane = threadIdx.x;
  const double a = A[(lane & 15) * 4 + (lane >> 4)];
  const double b = B[(lane >> 4) * 16 + (lane & 15)];
  dbl4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
}

bool gpis_ok(const cdx_gpis* g) {
  return g && g->X1 && g->alpha && g->N > 0 && g->N_pad >= g->N && g->N_pad % CDX_NPAD_ALIGN == 0 && g->kernel >= 0 &&
         g->kernel <= 2;
}

int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

}  // namespace

namespace cdx {

// Split-K chunk (K-steps) of the whitened pass, 0 = one workgroup per (query tile, stripe).  Used
// when those workgroups do not fill the 256 CUs (config 1: 4 workgroups of up to 23 serial K-steps):
// the largest power-of-two chunk ≥ 2 K-steps giving ≥ 256 units, within 256 MB of chunk partials.
static int var_chunk(const cdx_gpis& g, int64_t M) {
  const int Mt = (int)(round_up(M, ST_BM) / ST_BM), Nt = g.N_pad / ST_BN;
  if ((int64_t)Mt * Nt >= 256) return 0;
  auto units = [&](int c) {
    int u = 0;
    for (int nt = 0; nt < Nt; ++nt) u += (var_ksteps(nt, g.N, g.N_pad) + c - 1) / c;
    return (int64_t)Mt * u;
  };
  int c = 64;
  while (c > 2 && units(c) < 256) c >>= 1;
  const int64_t maxch = (var_ksteps(Nt - 1, g.N, g.N_pad) + c - 1) / c;
  if (maxch * round_up(M, ST_BM) * g.N_pad * (int64_t)sizeof(double) > ((int64_t)256 << 20)) return 0;
  return c;
}

// Chunk/stripe partials, then (VAR_KLOAD) the K* buffer at a 256-byte aligned offset.
static size_t var_partial_bytes(const cdx_gpis& g, int64_t M) {
  const int c = var_chunk(g, M);
  size_t b;
  if (c > 0) {
    const int Nt = g.N_pad / ST_BN;
    b = (size_t)((var_ksteps(Nt - 1, g.N, g.N_pad) + c - 1) / c) * (size_t)round_up(M, ST_BM) * g.N_pad * sizeof(double);
  } else {
    b = (size_t)(g.N_pad / ST_BN) * (size_t)round_up(M, ST_BM) * sizeof(double);
  }
  return (b + 255) / 256 * 256;
}

size_t gpis_var_ws_bytes(const cdx_gpis& g, int64_t M) {
  return var_partial_bytes(g, M) + (VAR_KLOAD ? (size_t)M * g.N_pad * sizeof(double) : 0);
}

// Pieces per query tile of the ∇std pass: one round of workgroups over the 256 CUs when the query
// tiles alone do not fill it (pieces of ≥ 4 K-steps), else one piece per tile.
static int gradv_parts(const cdx_gpis& g, int Mt) {
  int W = 0;
  for (int nt = 0; nt < g.N_pad / ST_BN; ++nt) W += gradv_ksteps(nt, g.N);
  int p = Mt >= 256 ? 1 : (256 + Mt - 1) / Mt;
  return std::max(1, std::min(p, W / 4));
}

size_t gpis_grad_ws_bytes(const cdx_gpis& g, int64_t M) {
  if (M <= 0) return 0;
  const int Mt = (int)(round_up(M, ST_BM) / ST_BM), Nt = g.N_pad / ST_BN;
  const size_t slots = (size_t)std::max(gradv_parts(g, Mt) + Nt, Nt);  // GRADV pieces + stripes; GRAD: stripes
  return slots * (size_t)round_up(M, ST_BM) * 4 * sizeof(double);
}

template <int KT>
static void var_launch_kt(const cdx_gpis& g, const double* X, int64_t M, double* std_out, double* var_out,
                          double* partial, int64_t M_pad, int Mt, int n_tiles, double* vout, hipStream_t s,
                          const VarSelect* vs) {
  const int64_t G = vs ? M / vs->T : 0;
  // Σ V² needs the K-summed V: a split-K launch (few query tiles) stores per-chunk V tiles and a
  // second kernel sums them in a fixed order (no atomics: deterministic).
  const int chunk = var_chunk(g, M);
  double* kstar = nullptr;
  if (VAR_KLOAD) {
    kstar = reinterpret_cast<double*>(reinterpret_cast<char*>(partial) + var_partial_bytes(g, M));
    hipLaunchKernelGGL(gpis_kstar_kernel<KT>, dim3((unsigned)((M + KS_ROWS - 1) / KS_ROWS)), dim3(256), 0, s, g, X, M,
                       kstar);
  }
  if (chunk > 0) {
    int units = 0;
    for (int nt = 0; nt < n_tiles; ++nt) units += (var_ksteps(nt, g.N, g.N_pad) + chunk - 1) / chunk;
    prof_mark(PROF_GPIS_STD, true, s);
    hipLaunchKernelGGL((gpis_std_kernel<KT, MODE_VAR>), dim3((unsigned)(Mt * units)), dim3(ST_THREADS), 0, s,
                       g, X, M, partial, M_pad, Mt, n_tiles, nullptr, kstar, nullptr, chunk, RefineList{});
    hipLaunchKernelGGL(gpis_var_splitk_finalize<KT>, dim3((unsigned)M), dim3(256), 0, s, g, partial, M_pad, chunk,
                       vout, std_out, var_out);
    prof_mark(PROF_GPIS_STD, false, s);
    if (vs)
      hipLaunchKernelGGL(gpis_select_kernel, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, s, G, vs->T,
                         (const double*)std_out, X, vs->sel, vs->Xg);
    return;
  }
  prof_mark(PROF_GPIS_STD, true, s);
  hipLaunchKernelGGL((gpis_std_kernel<KT, MODE_VAR>), dim3((unsigned)(Mt * n_tiles)), dim3(ST_THREADS), 0, s,
                     g, X, M, partial, M_pad, Mt, n_tiles, vout, kstar, nullptr, 0, RefineList{});
  prof_mark(PROF_GPIS_STD, false, s);
  if (vs && 256 % vs->T == 0) {
    hipLaunchKernelGGL(gpis_var_finalize_select<KT>, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, g, partial,
                       M, vs->T, M_pad, n_tiles, std_out, var_out, X, vs->sel, vs->Xg);
    return;
  }
  hipLaunchKernelGGL(gpis_var_finalize<KT>, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, g, partial, M, M_pad,
                     n_tiles, std_out, var_out);
  if (vs)
    hipLaunchKernelGGL(gpis_select_kernel, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, s, G, vs->T,
                       (const double*)std_out, X, vs->sel, vs->Xg);
}

template <int KT>
static void grad_launch_kt(const cdx_gpis& g, const double* X, int64_t M, const int64_t* sel, const double* var,
                           double* gstd, double* partial, int64_t M_pad, int Mt, int n_tiles, const double* vin,
                           hipStream_t s, const int64_t* vrow, GradFold* fold) {
  prof_mark(PROF_GPIS_GRAD, true, s);
  GradSlots slots;
  slots.n = 0;
  if (vin) {
    const int parts = gradv_parts(g, Mt);
    // cost-balanced pieces (gradv_cut): per-stripe costs to the kernel through the list's cost table
    GradCosts gc;
    RefineList rl{};
#if defined(CDX_GRAD_COSTCUT)  // off: 0.295 vs 0.286 ms for the ∇std pass (profiles/r03w_cuts_ab.jsonl)
    if (n_tiles <= GC_MAX_NT && n_tiles <= RC_MAX_NT) {
      gc.n = rl.n_uc = n_tiles;
      for (int nt = 0; nt < n_tiles; ++nt) gc.uc[nt] = rl.uc[nt] = gradv_unit_cost(nt, g.N);
    }
#endif
    // slot p + nt per (piece, stripe) segment the kernel runs (same cut as gpis_std_kernel<GRADV>)
    int W = 0;
    for (int nt = 0; nt < n_tiles; ++nt) W += gradv_ksteps(nt, g.N);
    for (int p = 0; p < parts; ++p) {
      const int q0 = gradv_cut(p, parts, W, g.N, n_tiles, gc.uc, gc.n),
                q1 = gradv_cut(p + 1, parts, W, g.N, n_tiles, gc.uc, gc.n);
      for (int nt = 0, s0 = 0; nt < n_tiles; ++nt) {
        const int s1 = s0 + gradv_ksteps(nt, g.N);
        if (std::max(q0, s0) < std::min(q1, s1) && slots.n < GRAD_MAX_SLOTS) slots.t[slots.n++] = (unsigned short)(p + nt);
        s0 = s1;
      }
    }
    hipLaunchKernelGGL((gpis_std_kernel<KT, MODE_GRADV>), dim3((unsigned)(Mt * parts)), dim3(ST_THREADS), 0,
                       s, g, X, M, partial, M_pad, Mt, n_tiles, nullptr, vin, vrow ? vrow : sel, parts, rl);
    if (fold) {  // the consumer sums the pieces itself (same slots in the same order as the list above)
      prof_mark(PROF_GPIS_GRAD, false, s);
      fold->partial = partial;
      fold->M_pad = M_pad;
      fold->parts = parts;
      fold->W = W;
      fold->Nt = n_tiles;
      fold->N = g.N;
      fold->gc = gc;
      fold->n_slots = 0;
#if !defined(CDX_FOLD_CUTS)  // (A/B: the consumer walks the cuts itself)
      if (slots.n <= GF_MAX_SLOTS) {
        fold->n_slots = slots.n;
        for (int i = 0; i < slots.n; ++i) fold->slot[i] = slots.t[i];
      }
#endif
      return;
    }
  } else {
    for (int nt = 0; nt < n_tiles && nt < GRAD_MAX_SLOTS; ++nt) slots.t[slots.n++] = (unsigned short)nt;
    hipLaunchKernelGGL((gpis_std_kernel<KT, MODE_GRAD>), dim3((unsigned)(Mt * n_tiles)), dim3(ST_THREADS), 0, s, g,
                       X, M, partial, M_pad, Mt, n_tiles, nullptr, nullptr, nullptr, 0, RefineList{});
  }
  prof_mark(PROF_GPIS_GRAD, false, s);
  hipLaunchKernelGGL(gpis_grad_finalize, dim3((unsigned)((M + 63) / 64)), dim3(64), 0, s, partial, M, M_pad,
                     slots, sel, var, gstd);
}

size_t gpis_v_bytes(const cdx_gpis& g, int64_t M) {
  return (size_t)round_up(M, ST_BM) * (size_t)g.N_pad * sizeof(double);
}

int gpis_var_launch(const cdx_gpis& g, const double* X, int64_t M, double* std_out, double* var_out, void* ws,
                    hipStream_t s, double* vout, const VarSelect* vs) {
  if (M <= 0) return CDX_OK;
  if (vs && (vs->T <= 0 || M % vs->T != 0 || !vs->sel || !vs->Xg)) return CDX_EINVAL;
  const int64_t M_pad = round_up(M, ST_BM);
  const int n_tiles = g.N_pad / ST_BN;
  if (M_pad / ST_BM * n_tiles > 0x7fffffff) return CDX_EINVAL;
  const int Mt = (int)(M_pad / ST_BM);
  double* partial = static_cast<double*>(ws);
  switch (g.kernel) {
    case CDX_KERNEL_TPS: var_launch_kt<CDX_KERNEL_TPS>(g, X, M, std_out, var_out, partial, M_pad, Mt, n_tiles, vout, s, vs); break;
    case CDX_KERNEL_RBF: var_launch_kt<CDX_KERNEL_RBF>(g, X, M, std_out, var_out, partial, M_pad, Mt, n_tiles, vout, s, vs); break;
    default: var_launch_kt<CDX_KERNEL_JOINT>(g, X, M, std_out, var_out, partial, M_pad, Mt, n_tiles, vout, s, vs); break;
  }
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int gpis_grad_launch(const cdx_gpis& g, const double* X, int64_t M, const int64_t* sel, const double* var,
                     double* gstd, void* ws, hipStream_t s, const double* vin, const int64_t* vrow, GradFold* fold) {
  if (vin && !g.Linv) return CDX_EINVAL;
  if (fold && !vin) return CDX_EINVAL;
  if (M <= 0) return CDX_OK;
  const int64_t M_pad = round_up(M, ST_BM);
  const int n_tiles = g.N_pad / ST_BN;
  if (M_pad / ST_BM * (int64_t)(256 + n_tiles) > 0x7fffffff) return CDX_EINVAL;
  if (256 + n_tiles > GRAD_MAX_SLOTS) return CDX_EINVAL;  // finalize slot list (N_pad ≤ 65 536)
  const int Mt = (int)(M_pad / ST_BM);
  double* partial = static_cast<double*>(ws);
  switch (g.kernel) {
    case CDX_KERNEL_TPS: grad_launch_kt<CDX_KERNEL_TPS>(g, X, M, sel, var, gstd, partial, M_pad, Mt, n_tiles, vin, s, vrow, fold); break;
    case CDX_KERNEL_RBF: grad_launch_kt<CDX_KERNEL_RBF>(g, X, M, sel, var, gstd, partial, M_pad, Mt, n_tiles, vin, s, vrow, fold); break;
    default: grad_launch_kt<CDX_KERNEL_JOINT>(g, X, M, sel, var, gstd, partial, M_pad, Mt, n_tiles, vin, s, vrow, fold); break;
  }
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

// Pieces of the refine pass: one per CU.
constexpr int REFINE_PIECES = 256;

// [stripe partials][cut-unit partial tiles][arrival counters]
static size_t refine_part_bytes(const cdx_gpis& g, int64_t Mcap) {
  return ((size_t)(g.N_pad / ST_BN) * (size_t)round_up(Mcap, ST_BM) * sizeof(double) + 255) / 256 * 256;
}
static size_t refine_slot_bytes() { return (size_t)REFINE_PIECES * 2 * ST_BM * ST_BN * sizeof(double); }
// (+1: the repair pass's workgroup arrival counter, after the cut-unit counters)
static size_t refine_cnt_bytes(const cdx_gpis& g, int64_t Mcap) {
  return ((size_t)(g.N_pad / ST_BN) * (size_t)(round_up(Mcap, ST_BM) / ST_BM) * sizeof(int) + sizeof(int) + 255) / 256 * 256;
}

static size_t refine_cuts_bytes() { return ((REFINE_PIECES + 1) * sizeof(int64_t) + 255) / 256 * 256; }

size_t gpis_refine_ws_bytes(const cdx_gpis& g, int64_t Mcap) {
  return refine_part_bytes(g, Mcap) + refine_slot_bytes() + refine_cnt_bytes(g, Mcap) + refine_cuts_bytes();
}

int gpis_refine_reset(const cdx_gpis& g, int64_t Mcap, void* ws, hipStream_t s) {
  char* c = static_cast<char*>(ws) + refine_part_bytes(g, Mcap) + refine_slot_bytes();
  return hipMemsetAsync(c, 0, refine_cnt_bytes(g, Mcap), s) == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

template <int KT>
static void refine_launch_kt(const cdx_gpis& g, const double* X, int64_t Mcap, const RefineList& rl, double* partial,
                             int64_t M_pad, double* vout, hipStream_t s, bool prof, hipEvent_t after) {
  if (prof) prof_mark(PROF_GPIS_STD, true, s);
  hipLaunchKernelGGL((gpis_std_kernel<KT, MODE_VARL>), dim3(REFINE_PIECES), dim3(ST_THREADS), 0, s, g, X, Mcap, partial,
                     M_pad, 0, g.N_pad / ST_BN, vout, nullptr, nullptr, 0, rl);
  if (prof) prof_mark(PROF_GPIS_STD, false, s);
  if (after) (void)hipEventRecord(after, s);
#if !defined(CDX_MERGE_FUSED)
  if (!rl.rs.on)  // (the repair pass runs whole units: nothing to merge)
    hipLaunchKernelGGL(gpis_var_merge, dim3(REFINE_PIECES), dim3(MERGE_THREADS), 0, s, g, rl, M_pad, partial, vout);
#endif
}

int gpis_refine_launch(const cdx_gpis& g, const double* X, const int* rows, const int* extra, int G, int64_t Mcap,
                       void* ws, double* vout, hipStream_t s, double** partial_out, int64_t* M_pad_out, const int* gate,
                       bool prof, hipEvent_t after_refine, const RepairSel* repair) {
  if (Mcap <= 0 || G <= 0 || G > Mcap) return CDX_EINVAL;
  if (repair && (!gate || rows || extra || repair->G * repair->T != G || repair->stats != gate)) return CDX_EINVAL;
  const int64_t M_pad = round_up(Mcap, ST_BM);
  double* partial = static_cast<double*>(ws);
  char* slots = static_cast<char*>(ws) + refine_part_bytes(g, Mcap);
  RefineList rl{rows, extra, G, reinterpret_cast<double*>(slots), reinterpret_cast<int*>(slots + refine_slot_bytes()),
                (int)(M_pad / ST_BM),
                reinterpret_cast<int64_t*>(slots + refine_slot_bytes() + refine_cnt_bytes(g, Mcap)), 0, {}, gate, {}};
  if (repair) {
    rl.rs = *repair;
    rl.rs.on = true;
    rl.rs.done = rl.cnt + (size_t)(g.N_pad / ST_BN) * (size_t)(M_pad / ST_BM);
  }
  const int Nt = g.N_pad / ST_BN;
  if (Nt <= RC_MAX_NT) {
    rl.n_uc = Nt;
    for (int nt = 0; nt < Nt; ++nt) rl.uc[nt] = var_unit_cost(nt, g.N, g.N_pad);
  }
  switch (g.kernel) {
    case CDX_KERNEL_TPS: refine_launch_kt<CDX_KERNEL_TPS>(g, X, Mcap, rl, partial, M_pad, vout, s, prof, after_refine); break;
    case CDX_KERNEL_RBF: refine_launch_kt<CDX_KERNEL_RBF>(g, X, Mcap, rl, partial, M_pad, vout, s, prof, after_refine); break;
    default: refine_launch_kt<CDX_KERNEL_JOINT>(g, X, Mcap, rl, partial, M_pad, vout, s, prof, after_refine); break;
  }
  if (partial_out) *partial_out = partial;
  if (M_pad_out) *M_pad_out = M_pad;
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

}  // namespace cdx

extern "C" {

int cdx_gpis_mean(const cdx_gpis* g, const double* X, int64_t M, double* mean, double* grad_mean, double* normal,
                  cdx_stream_t stream) {
  if (!gpis_ok(g)) return g && (g->kernel < 0 || g->kernel > 2) ? CDX_EKERNEL : CDX_EINVAL;
  if (M < 0 || (M > 0 && (!X || !mean))) return CDX_EINVAL;
  if (M == 0) return CDX_OK;
  const dim3 grid((unsigned)((M + MEAN_Q - 1) / MEAN_Q));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  cdx::prof_mark(cdx::PROF_GPIS_MEAN, true, s);
  switch (g->kernel) {
    case CDX_KERNEL_TPS:
#if !defined(CDX_MEAN_DIRECT) && CDX_MEAN_QPT > 1
      hipLaunchKernelGGL(gpis_mean_tps_blocked_kernel, dim3((unsigned)((M + MQ_PER_WG - 1) / MQ_PER_WG)), dim3(MEAN_BLOCK), 0, s,
                         *g, X, M, mean, grad_mean, normal);
#else
      hipLaunchKernelGGL(gpis_mean_kernel<CDX_KERNEL_TPS>, grid, dim3(MEAN_BLOCK), 0, s, *g, X, M, mean, grad_mean, normal);
#endif
      break;
    case CDX_KERNEL_RBF: hipLaunchKernelGGL(gpis_mean_kernel<CDX_KERNEL_RBF>, grid, dim3(MEAN_BLOCK), 0, s, *g, X, M, mean, grad_mean, normal); break;
    default: hipLaunchKernelGGL(gpis_mean_kernel<CDX_KERNEL_JOINT>, grid, dim3(MEAN_BLOCK), 0, s, *g, X, M, mean, grad_mean, normal); break;
  }
  cdx::prof_mark(cdx::PROF_GPIS_MEAN, false, s);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

size_t cdx_gpis_std_workspace(const cdx_gpis* g, int64_t M) {
  if (!g || M <= 0 || g->N_pad <= 0) return 0;
  return cdx::gpis_var_ws_bytes(*g, M) + cdx::gpis_grad_ws_bytes(*g, M) + (size_t)round_up(M, 32) * sizeof(double) +
         cdx::gpis_v_bytes(*g, M);
}

int cdx_gpis_std(const cdx_gpis* g, const double* X, int64_t M, double* std_out, double* grad_std, void* workspace,
                 cdx_stream_t stream) {
  if (!gpis_ok(g) || !g->Ainv || !g->Linv_t) return g && (g->kernel < 0 || g->kernel > 2) ? CDX_EKERNEL : CDX_EINVAL;
  if (M < 0 || (M > 0 && (!X || !std_out || !workspace))) return CDX_EINVAL;
  if (M == 0) return CDX_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* ws = static_cast<char*>(workspace);
  double* var = reinterpret_cast<double*>(ws);
  void* pv = ws + (size_t)round_up(M, 32) * sizeof(double);
  void* pg = static_cast<char*>(pv) + cdx::gpis_var_ws_bytes(*g, M);
  double* V = reinterpret_cast<double*>(static_cast<char*>(pg) + cdx::gpis_grad_ws_bytes(*g, M));
  const bool whitened_grad = grad_std && g->Linv;  // ∇std = −L⁻ᵀv·∇k/std from the kept V
  int rc = cdx::gpis_var_launch(*g, X, M, std_out, var, pv, s, whitened_grad ? V : nullptr);
  if (rc || !grad_std) return rc;
  return cdx::gpis_grad_launch(*g, X, M, nullptr, var, grad_std, pg, s, whitened_grad ? V : nullptr);
}

#if defined(CDX_DIAG_WGTIME)
int cdx_diag_wgtime(void* host_out, int n) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(cdx_wgtime), (size_t)n * 32, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? CDX_OK : CDX_ELAUNCH;
}
#endif

// Test hook: D[16×16] = A[16×4]·B[4×16] through one v_mfma_f64_16x16x4_f64 (layout check).
int cdx_selftest_mfma_f64(const double* A, const double* B, double* D, cdx_stream_t stream) {
  if (!A || !B || !D) return CDX_EINVAL;
  hipLaunchKernelGGL(mfma_f64_selftest_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), A, B, D);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

}  // extern "C"
