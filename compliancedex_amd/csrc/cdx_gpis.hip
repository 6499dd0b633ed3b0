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

#include <type_traits>

#include "cdx_gpis.h"
#include "cdx_gpis_launch.h"
#include "cdx_prof.h"

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
constexpr int MEAN_Q = 16, MEAN_SPLIT = 16, MEAN_BLOCK = MEAN_Q * MEAN_SPLIT;

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
// W = K*·E11⁻¹ tile of 128 queries × 256 output columns per 512-thread workgroup (one per CU),
// K-step 16, two LDS buffers (register-staged: the K* tile is computed, not loaded), one barrier
// per K-step.  Waves form a 2×4 grid; each owns 64×64 = 4×4 v_mfma_f64_16x16x4_f64 tiles.  The
// 256-wide tile halves the per-output-column cost of generating K* on chip against the 128-wide
// tile of 2×2 waves (-DCDX_STD_WN2): 2.41 vs 2.58 ms at M = 16 384, N = 2000.
// Fragment maps (cdna_hip_programming.md §3, f64 form):
//   A: lane l holds A[row l&15][k l>>4];  B: B[k l>>4][col l&15]
//   C/D: reg r of lane l is D[row (l>>4) + 4r][col l&15]
// LDS rows are padded to 144 doubles (row stride ≡ 32 dwords mod 64): the two half-waves of a
// ds_read_b64 (rows k, k+1) land on disjoint banks.
constexpr int ST_BM = 128, ST_BK = 16, ST_LD = 144;
constexpr int ST_TILE = ST_BK * ST_LD;                          // doubles per staged K* tile
#if defined(CDX_STD_WN2)
constexpr int ST_WN = 2;                                        // waves along N (2 or 4)
#else
constexpr int ST_WN = 4;
#endif
static_assert(CDX_NPAD_ALIGN % (64 * ST_WN) == 0, "N_pad alignment must cover the tile width");
constexpr int ST_BN = 64 * ST_WN;                               // output columns per workgroup
constexpr int ST_THREADS = 128 * ST_WN;                         // 2 row-waves × ST_WN column-waves
constexpr int ST_LDB = ST_BN + 16;                              // padded E11⁻¹ row (≡ 32 dwords mod 64)
constexpr int ST_BTILE = ST_BK * ST_LDB;
constexpr int ST_SMEM = 2 * (ST_TILE + ST_BTILE) + ST_BM * 3;   // 2 buffers × (K*, E11⁻¹) + query tile

// T4 layout of the B tile (v_mfma_f64_4x4x4_4b_f64 path, triangular modes): lane l needs
// B[k = l>>4][wc + 4·cg + (l&3)] for cg = 0..15, so each 64-column wave slice is stored as
// [j = col&3][cg = col>>2 (16) + 2 pad] (72 doubles) and rows are T4_LDB ≡ 8 (mod 32) doubles
// apart: the 16 (k, j) lane groups of a ds_read_b128 then cover all 64 banks (the 4 β lanes of a
// group read the same address: broadcast).
constexpr int T4_SLICE = 72;
constexpr int T4_LDB = 4 * T4_SLICE + 8;                          // 296
constexpr int T4_BTILE = ST_BK * T4_LDB;
constexpr int T4_SMEM = 2 * (ST_TILE + T4_BTILE) + ST_BM * 3;
__device__ __forceinline__ int t4_bpos(int c) { return (c >> 6) * T4_SLICE + (c & 3) * 18 + ((c & 63) >> 2); }

typedef double dbl2v __attribute__((ext_vector_type(2)));

// v2: 128 queries × ST_BN output columns per workgroup of 2 × ST_WN waves, each wave owning
// 64×64 = 4×4 v_mfma_f64_16x16x4_f64 tiles; K-step 16, two LDS buffers, one barrier per step.
//
// MODE_GRAD (∇std, explicit inverse): A = K* (generated), B = E11⁻¹, W = K*·E11⁻¹, epilogue
//   Σ W·k and Σ W·kd·(x − x_n) → 4 partials per (column tile, query).
// MODE_VAR (std, whitened): A = K* (generated), B = L⁻ᵀ (upper triangular), V = K*·L⁻ᵀ =
//   (L⁻¹K*ᵀ)ᵀ, epilogue Σ V² → 1 partial per (column tile, query); optionally V itself is stored
//   (vout, [M_pad, N_pad]).  Column tile nt only needs K-rows j < n0 + ST_BN (and < N).
// MODE_GRADV (∇std from the stored whitened vector): A = V rows (loaded, row vsel[m] of vin),
//   B = L⁻¹ (lower triangular), W = V·L⁻¹ = (L⁻ᵀv)ᵀ = (E11⁻¹k)ᵀ, the MODE_GRAD epilogue (linear
//   in W, so K can be split).  Column tile nt only needs K-rows i ≥ n0: N² flops per query
//   instead of 2N²; launched split-K over 256-row chunks (Nt(Nt+1)/2 partial slots).
// The triangular modes' tile costs run 1..Nt K-sweeps: stripes are paired heavy+light per XCD.
enum { MODE_GRAD = 0, MODE_VAR = 1, MODE_GRADV = 2 };
// MFMA shape per pass (profiles/r01x_std_variants.jsonl, r01y_gradv_ab.txt): the whitened std pass
// runs equally fast on 16x16x4 and 4x4x4_4b (1.30 ms at M = 16 384); the ∇std pass is faster on
// 4x4x4_4b for contiguous queries (0.37 vs 0.43 ms at M = 4096) but slower on the closure's gathered
// argmax rows (0.53 vs 0.44 ms): 16x16x4 by default, 4x4x4_4b for both behind -DCDX_STD_T4.
#if defined(CDX_STD_T4) && !defined(CDX_STD_WN2)
constexpr bool STD_T4 = true, GRADV_T4 = true;
#else
constexpr bool STD_T4 = false, GRADV_T4 = false;
#endif


// K-range [lo, hi) of stripe nt in the triangular modes.
__device__ __host__ inline void stripe_k_range(int mode, int nt, int N, int& lo, int& hi) {
  lo = mode == MODE_GRADV ? nt * ST_BN : 0;
  hi = mode == MODE_GRADV ? N : min(N, nt * ST_BN + ST_BN);
}

// Split-K units per query tile: stripe nt contributes ceil((hi − lo)/CH) chunks of CH rows.
__host__ inline int split_units(int mode, int Nt, int N, int CH) {
  int u = 0;
  for (int nt = 0; nt < Nt; ++nt) {
    int lo, hi;
    stripe_k_range(mode, nt, N, lo, hi);
    u += hi > lo ? (hi - lo + CH - 1) / CH : 0;
  }
  return u;
}

// ksplit = 0: one workgroup per (query tile, stripe).  ksplit = s > 0 (GRADV): one workgroup per
// (query tile, stripe, K-chunk of ST_BN/s rows), `upm` units per query tile, one partial slot per
// unit (summed in a fixed order by the finalize kernel: deterministic).
template <int KT, int MODE, bool T4 = false>
__global__ __launch_bounds__(ST_THREADS, 8 / ST_WN) void gpis_std_kernel(cdx_gpis g, const double* __restrict__ X,
                                                                        int64_t M, double* __restrict__ partial,
                                                                        int64_t M_pad, int Mt, int Nt,
                                                                        double* __restrict__ vout,
                                                                        const double* __restrict__ vin,
                                                                        const int64_t* __restrict__ vsel, int ksplit,
                                                                        int upm) {
  constexpr bool VAR = MODE == MODE_VAR;
  constexpr bool TRI = MODE != MODE_GRAD;
  static_assert(!T4 || (TRI && ST_WN == 4), "the 4x4x4 path covers the triangular modes of the 128x256 tile");
  constexpr int LDB = T4 ? T4_LDB : ST_LDB;
  constexpr int BTILE = T4 ? T4_BTILE : ST_BTILE;
  __shared__ __attribute__((aligned(16))) double smem[T4 ? T4_SMEM : ST_SMEM];
  double* xq = smem + 2 * (ST_TILE + BTILE);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = Mt * Nt;
  const int b = blockIdx.x;
  int nt, mt, pslot, kbeg_ = 0, kend_ = g.N;
  const bool split = ksplit > 0;
  if (TRI && split) {
    // Split-K: unit = (stripe nt, K-chunk c) so units cost about the same (the ∇std pass runs on
    // E·L_q queries only; small-M std passes would otherwise run few, long workgroups).  Units of
    // one (nt, c) block share their B block: each XCD takes a contiguous run of blocks over all
    // query tiles.  Partial slot = block index.
    const int CH = ST_BN / ksplit;
    const int U = Mt * upm;
    const int t = (U & 7) == 0 ? (b & 7) * (U >> 3) + (b >> 3) : b;
    int blk = t / Mt;
    mt = t - blk * Mt;
    pslot = blk;
    for (nt = 0;; ++nt) {
      int lo, hi;
      stripe_k_range(MODE, nt, g.N, lo, hi);
      const int nch = hi > lo ? (hi - lo + CH - 1) / CH : 0;
      if (blk < nch) {
        kbeg_ = lo + blk * CH;
        kend_ = min(hi, kbeg_ + CH);
        break;
      }
      blk -= nch;
    }
  } else if (TRI) {
    // Stripe nt costs ∝ nt + 1 K-sweeps (VAR; GRADV: Nt − nt, mirrored below).  Pair stripes
    // (Nt−1−a, a) — every pair costs Nt + 1 — and
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
    pslot = nt;
  } else {
    // XCD-aware order: blocks b and b+8 share an XCD (round-robin dispatch); give each XCD a
    // contiguous run of n-major tiles so its L2 serves the same E11⁻¹ column stripes.
    const int t = (T & 7) == 0 ? (b & 7) * (T >> 3) + (b >> 3) : b;
    nt = t / Mt;
    mt = t - nt * Mt;
    pslot = nt;
  }
  const int64_t m0 = (int64_t)mt * ST_BM;
  const int n0 = nt * ST_BN;
  const int Np = g.N_pad;
  const double* __restrict__ Bop = MODE == MODE_VAR ? g.Linv_t : (MODE == MODE_GRADV ? g.Linv : g.Ainv);
  const double R = g.R, inv_s2 = 1.0 / (g.sigma * g.sigma);

  // K* generation: thread → query row gm, GEN_PER k-columns starting at gk (wave-uniform)
  constexpr int GEN_PER = ST_BM * ST_BK / ST_THREADS;  // 8 (2 col-waves) or 4 (4 col-waves)
  const int gm = tid & (ST_BM - 1);
  const int gk = __builtin_amdgcn_readfirstlane((tid >> 7) * GEN_PER);
  double qx, qy, qz;
  const double* vrow = nullptr;  // MODE_GRADV: this thread's row of the stored V
  {
    const int64_t m = min(m0 + gm, M - 1);  // pad rows replicate a valid query
    qx = X[3 * m]; qy = X[3 * m + 1]; qz = X[3 * m + 2];
    if (tid < ST_BM) { xq[3 * tid] = qx; xq[3 * tid + 1] = qy; xq[3 * tid + 2] = qz; }
    if (MODE == MODE_GRADV) vrow = vin + (vsel ? vsel[m] : m) * (int64_t)Np;
  }
  // B tile: 16 rows × ST_BN columns; thread → row ar, four 2-double pieces at columns ac + i·BSTR.
  // Interleaved pieces keep each ds_write_b128 conflict-free (16 consecutive lanes cover the 64
  // banks once; 8 consecutive doubles per thread made it 4-way conflicted, ≈9 % of the K-step)
  // and each global load a contiguous 16 B × 32 lanes.
  constexpr int A_TPR = ST_BN / 8;                      // threads per row
  constexpr int BSTR = 2 * A_TPR;                       // doubles between a thread's pieces
  const int ar = tid / A_TPR, ac = (tid % A_TPR) * 2;
  // wave → 64×64 sub-tile.  With 4 column waves, waves w and w+4 share SIMD w%4 (round-robin wave
  // placement); giving them complementary columns (w, 7−w) lets the triangular modes skip the
  // all-zero K-steps of the diagonal block per wave without idling a SIMD (see skip_mfma below).
  const int cwave = ST_WN == 4 ? (wave < 4 ? wave : 7 - wave) : wave % ST_WN;
  const int wr = (wave / ST_WN) * 64, wc = __builtin_amdgcn_readfirstlane(cwave * 64);

  dbl2v av[4];
  double kv[GEN_PER];
  auto stage_load = [&](int kb) {
    const dbl2v* src = reinterpret_cast<const dbl2v*>(Bop + (int64_t)(kb + ar) * Np + n0 + ac);
#pragma unroll
    for (int i = 0; i < 4; ++i) av[i] = src[i * (BSTR / 2)];
    if (MODE == MODE_GRADV) {
#pragma unroll
      for (int i = 0; i < GEN_PER; ++i) {
#if defined(CDX_DIAG_NOVLOAD)  // timing-only diagnostic build: outputs are wrong
        kv[i] = qx + i;
#else
        kv[i] = vrow[kb + gk + i];
#endif
      }
      return;
    }
    const double* x1 = g.X1 + 3 * (kb + gk);
#pragma unroll
    for (int i = 0; i < GEN_PER; ++i) {
      const double dx = qx - x1[3 * i], dy = qy - x1[3 * i + 1], dz = qz - x1[3 * i + 2];
      double kd;
      gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, kv[i], kd);
    }
  };
  auto stage_write = [&](int buf) {
    double* Kt = smem + buf * (ST_TILE + BTILE);
    double* As = Kt + ST_TILE;
#pragma unroll
    for (int i = 0; i < GEN_PER; ++i) Kt[(gk + i) * ST_LD + gm] = kv[i];
    if constexpr (T4) {
      double* row = As + ar * LDB;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        row[t4_bpos(ac + BSTR * i)] = av[i].x;
        row[t4_bpos(ac + BSTR * i + 1)] = av[i].y;
      }
    } else {
      dbl2v* dst = reinterpret_cast<dbl2v*>(As + ar * LDB + ac);
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i * (BSTR / 2)] = av[i];
    }
  };

  dbl4 acc[4][4];      // 16x16x4 path: [row block][col block] of 16×16
  double acc4[4][16];  // T4 path: [row group rg (16 rows)][col group cg (4 cols)]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0, 0, 0, 0};
  if constexpr (T4) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc4[i][j] = 0.0;
  }

  // B rows ≥ N are zero: stop at the last live K-step; L⁻ᵀ (VAR) also stops at the tile's
  // diagonal, L⁻¹ (GRADV) starts there
  const int kbeg = split ? kbeg_ : 0;
  const int kend = split ? kend_ : (VAR ? min(g.N, n0 + ST_BN) : g.N);
  const int nK = (kend - kbeg + ST_BK - 1) / ST_BK;
  stage_load(kbeg);
  stage_write(0);
  __syncthreads();
  for (int s = 0; s < nK; ++s) {
    // Stage s+1 (clamped at the end: the extra stage lands in the buffer nobody reads again).
    const int kn = kbeg + (s + 1 < nK ? s + 1 : s) * ST_BK;
    {
      const dbl2v* src = reinterpret_cast<const dbl2v*>(Bop + (int64_t)(kn + ar) * Np + n0 + ac);
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = src[i * (BSTR / 2)];
      if (MODE == MODE_GRADV) {
#pragma unroll
        for (int i = 0; i < GEN_PER; ++i) {
#if defined(CDX_DIAG_NOVLOAD)  // timing-only diagnostic build: outputs are wrong
          kv[i] = qx + i + kn;
#else
          kv[i] = vrow[kn + gk + i];
#endif
        }
      }
    }
    const double* x1 = g.X1 + 3 * (kn + gk);
    const double* Kt = smem + (s & 1) * (ST_TILE + BTILE);
    const double* As = Kt + ST_TILE;
    // This wave's B columns [n0 + wc, n0 + wc + 64) are all zero for the whole K-step when the step
    // lies past their diagonal (L⁻ᵀ, VAR) or before it (L⁻¹, GRADV): skip the MFMAs, keep the
    // staging and barriers.  acc + 0·A is acc, so results are bit-identical.
    const int kb = kbeg + s * ST_BK;
    const bool skip_mfma = (MODE == MODE_VAR && kb >= n0 + wc + 64) || (MODE == MODE_GRADV && kb + ST_BK <= n0 + wc);
    auto kstep4 = [&](auto do_mfma) {  // v_mfma_f64_4x4x4_4b_f64: 16 rows × 4 cols × 4 deep per issue
#pragma unroll
      for (int kk = 0; kk < ST_BK; kk += 4) {
        const int kra = (kk + (lane >> 4)) * ST_LD + (lane & 15);
        double a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = Kt[kra + wr + 16 * i];
        const dbl2v* bp = reinterpret_cast<const dbl2v*>(As + (kk + (lane >> 4)) * LDB + cwave * T4_SLICE +
                                                         (lane & 3) * 18);
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // B fragments in two halves of 8 column groups (register budget)
          double bb[8];
#pragma unroll
          for (int c = 0; c < 4; ++c) { const dbl2v v = bp[4 * h + c]; bb[2 * c] = v.x; bb[2 * c + 1] = v.y; }
          if constexpr (decltype(do_mfma)::value) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int j = 0; j < 8; ++j)
                acc4[i][8 * h + j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[i], bb[j], acc4[i][8 * h + j], 0, 0, 0);
          }
        }
#pragma unroll
        for (int i = kk * GEN_PER / ST_BK; i < (kk + 4) * GEN_PER / ST_BK; ++i) {
          if (MODE == MODE_GRADV) break;  // loaded, not generated
#if defined(CDX_DIAG_NOGEN)  // timing-only diagnostic build: outputs are wrong
          kv[i] = qx - x1[3 * i];
#else
          const double dx = qx - x1[3 * i], dy = qy - x1[3 * i + 1], dz = qz - x1[3 * i + 2];
          double kd;
          gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, kv[i], kd);
#endif
        }
#if defined(CDX_STD_SCHED)
        if constexpr (decltype(do_mfma)::value) {
          __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // fragment reads first
#pragma unroll
          for (int q = 0; q < 64; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // then one VALU
          }
        }
#endif
      }
    };
    // 16x16x4 K-step: four 4-deep substeps of 16 MFMAs; the next substep's 8 fragment reads are
    // issued ahead of this substep's MFMAs (register double buffer), so only the first substep
    // after the barrier waits on LDS latency.
    auto kstep = [&](auto do_mfma) {
      double fa[2][4], fb[2][4];
      auto frag = [&](int kk, double* a, double* bb) {
        const int kra = (kk + (lane >> 4)) * ST_LD + (lane & 15);
        const int krb = (kk + (lane >> 4)) * ST_LDB + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) { a[i] = Kt[kra + wr + 16 * i]; bb[i] = As[krb + wc + 16 * i]; }
      };
      if constexpr (decltype(do_mfma)::value) frag(0, fa[0], fb[0]);
#pragma unroll
      for (int kk = 0; kk < ST_BK; kk += 4) {
        const int cur = (kk >> 2) & 1;
        if constexpr (decltype(do_mfma)::value) {
          if (kk + 4 < ST_BK) frag(kk + 4, fa[cur ^ 1], fb[cur ^ 1]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
#if defined(CDX_DIAG_NOMFMA)  // timing-only diagnostic build: outputs are wrong
            acc[i][j][0] += fa[cur][i] * fb[cur][j];
#else
            if constexpr (decltype(do_mfma)::value)
              acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0);
#endif
          }
        // K* of the next stage spread over the four 16-MFMA groups (overlaps the matrix pipe)
#pragma unroll
        for (int i = kk * GEN_PER / ST_BK; i < (kk + 4) * GEN_PER / ST_BK; ++i) {
          if (MODE == MODE_GRADV) break;  // loaded, not generated
#if defined(CDX_DIAG_NOGEN)  // timing-only diagnostic build: outputs are wrong
          kv[i] = qx - x1[3 * i];
#else
          const double dx = qx - x1[3 * i], dy = qy - x1[3 * i + 1], dz = qz - x1[3 * i + 2];
          double kd;
          gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, kv[i], kd);
#endif
        }
#if defined(CDX_STD_SCHED)
        if constexpr (decltype(do_mfma)::value) {
          if (kk + 4 < ST_BK) __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // next substep's reads first
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // then up to four VALU
          }
        }
#endif
      }
    };
    if constexpr (T4) {
      if (skip_mfma) kstep4(std::false_type{});
      else kstep4(std::true_type{});
    } else {
      if (skip_mfma) kstep(std::false_type{});
      else kstep(std::true_type{});
    }
    stage_write((s + 1) & 1);
    __syncthreads();
  }

  if constexpr (VAR) {
    // Epilogue: per owned row Σ V² over this wave's 64 columns, reduced over the 16 lanes of a
    // row, then over the column waves in LDS; V itself to vout when asked (16 lanes of a row write
    // 128 contiguous bytes).
    double* red = smem;  // [ST_WN][ST_BM]
    if constexpr (T4) {
      // lane l holds, for row group rg and column group cg, V[row][col] with
      // row = wr + 16·rg + 4·((l>>2)&3) + (l>>4), col = wc + 4·cg + (l&3)
      const int r4 = 4 * ((lane >> 2) & 3) + (lane >> 4);
      if (vout) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double* vr = vout + (m0 + wr + 16 * i + r4) * (int64_t)Np + n0 + wc + (lane & 3);
#pragma unroll
          for (int j = 0; j < 16; ++j) vr[4 * j] = acc4[i][j];
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double v = 0.0;
#pragma unroll
        for (int j = 0; j < 16; ++j) v = fma(acc4[i][j], acc4[i][j], v);
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        if ((lane & 3) == 0) red[cwave * ST_BM + wr + 16 * i + r4] = v;
      }
      __syncthreads();
      if (tid < ST_BM) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < ST_WN; ++w) v += red[w * ST_BM + tid];
        partial[(int64_t)pslot * M_pad + m0 + tid] = v;
      }
      return;
    }
    if (vout) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double* vr = vout + (m0 + wr + 16 * i + (lane >> 4) + 4 * r) * (int64_t)Np + n0 + wc + (lane & 15);
#pragma unroll
          for (int j = 0; j < 4; ++j) vr[16 * j] = acc[i][j][r];
        }
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
    return;
  }

  if constexpr (T4) {  // GRADV on the 4x4x4 layout (see the VAR epilogue for the lane map)
    double* red = smem;
    const int r4 = 4 * ((lane >> 2) & 3) + (lane >> 4);
    double ps[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ps[i][0] = ps[i][1] = ps[i][2] = ps[i][3] = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = n0 + wc + 4 * j + (lane & 3);
      const double nx = g.X1[3 * n], ny = g.X1[3 * n + 1], nz = g.X1[3 * n + 2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wr + 16 * i + r4;
        const double dx = xq[3 * row] - nx, dy = xq[3 * row + 1] - ny, dz = xq[3 * row + 2] - nz;
        double k, kd;
        gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, k, kd);
        const double w = acc4[i][j];
        const double wkd = w * kd;
        ps[i][0] += w * k;
        ps[i][1] += wkd * dx;
        ps[i][2] += wkd * dy;
        ps[i][3] += wkd * dz;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        double v = ps[i][c];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        ps[i][c] = v;
      }
    if ((lane & 3) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) red[(cwave * ST_BM + wr + 16 * i + r4) * 4 + c] = ps[i][c];
    }
    __syncthreads();
    for (int idx = tid; idx < ST_BM * 4; idx += ST_THREADS) {
      const int row = idx >> 2, c = idx & 3;
      double v = 0.0;
#pragma unroll
      for (int w = 0; w < ST_WN; ++w) v += red[(w * ST_BM + row) * 4 + c];
      partial[((int64_t)pslot * M_pad + m0 + row) * 4 + c] = v;
    }
    return;
  }

  // Epilogue: per owned row, s = Σ_n W k and g = Σ_n W kd (x_m − x_n) over this wave's 64 columns,
  // reduced over the 16 lanes of a row (xor-shuffles), then over the column waves in LDS.
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
        const double w = acc[i][j][r];
        const double wkd = w * kd;
        ps[r][0] += w * k;
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

// ∇std = −sign(v)·(Σ_n W kd (x − x_n))/sqrt|v| at query m, written to row sel[m] (identity when
// sel is null) with v = var[sel[m]] from the whitened pass.
__global__ __launch_bounds__(256) void gpis_grad_finalize(const double* __restrict__ partial, int64_t M,
                                                          int64_t M_pad, int n_tiles, const int64_t* __restrict__ sel,
                                                          const double* __restrict__ var, double* __restrict__ gstd) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  double g0 = 0, g1 = 0, g2 = 0;
  for (int t = 0; t < n_tiles; ++t) {
    const double* p = partial + ((int64_t)t * M_pad + m) * 4;
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

size_t gpis_var_ws_bytes(const cdx_gpis& g, int64_t M) {
  return (size_t)(g.N_pad / ST_BN) * (size_t)round_up(M, ST_BM) * sizeof(double);
}

// Split factor: the smallest s ∈ {1, 2, 4, 8, 16} giving ≥ 2 units per CU (256 CUs), else 16.
static int choose_split(int mode, const cdx_gpis& g, int64_t M) {
  const int Mt = (int)(round_up(M, ST_BM) / ST_BM), Nt = g.N_pad / ST_BN;
  int s = 1;
  while (s < 16 && (int64_t)Mt * split_units(mode, Nt, g.N, ST_BN / s) < 512) s *= 2;
  return s;
}

size_t gpis_grad_ws_bytes(const cdx_gpis& g, int64_t M) {
  if (M <= 0) return 0;
  const int s = choose_split(MODE_GRADV, g, M);
  const size_t upm = (size_t)split_units(MODE_GRADV, g.N_pad / ST_BN, g.N, ST_BN / s);
  const size_t dense = (size_t)(g.N_pad / ST_BN);  // the explicit-inverse pass's partial slots
  return (upm > dense ? upm : dense) * (size_t)round_up(M, ST_BM) * 4 * sizeof(double);
}

template <int KT>
static void var_launch_kt(const cdx_gpis& g, const double* X, int64_t M, double* std_out, double* var_out,
                          double* partial, int64_t M_pad, int Mt, int n_tiles, double* vout, hipStream_t s) {
  // (no split-K here: Σ V² needs the K-summed V, and summing chunk partials with atomics made the
  // result depend on arrival order — the std pass stays one workgroup per (query tile, stripe))
  prof_mark(PROF_GPIS_STD, true, s);
  hipLaunchKernelGGL((gpis_std_kernel<KT, MODE_VAR, STD_T4>), dim3((unsigned)(Mt * n_tiles)), dim3(ST_THREADS), 0, s,
                     g, X, M, partial, M_pad, Mt, n_tiles, vout, nullptr, nullptr, 0, 0);
  prof_mark(PROF_GPIS_STD, false, s);
  hipLaunchKernelGGL(gpis_var_finalize<KT>, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, g, partial, M, M_pad,
                     n_tiles, std_out, var_out);
}

template <int KT>
static void grad_launch_kt(const cdx_gpis& g, const double* X, int64_t M, const int64_t* sel, const double* var,
                           double* gstd, double* partial, int64_t M_pad, int Mt, int n_tiles, const double* vin,
                           hipStream_t s) {
  prof_mark(PROF_GPIS_GRAD, true, s);
  int n_parts = n_tiles;
  if (vin) {
    const int ks = choose_split(MODE_GRADV, g, M);
    n_parts = split_units(MODE_GRADV, n_tiles, g.N, ST_BN / ks);  // split-K units (stripe, K-chunk)
    hipLaunchKernelGGL((gpis_std_kernel<KT, MODE_GRADV, GRADV_T4>), dim3((unsigned)(Mt * n_parts)), dim3(ST_THREADS), 0,
                       s, g, X, M, partial, M_pad, Mt, n_tiles, nullptr, vin, sel, ks, n_parts);
  } else {
    hipLaunchKernelGGL((gpis_std_kernel<KT, MODE_GRAD>), dim3((unsigned)(Mt * n_tiles)), dim3(ST_THREADS), 0, s, g,
                       X, M, partial, M_pad, Mt, n_tiles, nullptr, nullptr, nullptr, 0, 0);
  }
  prof_mark(PROF_GPIS_GRAD, false, s);
  hipLaunchKernelGGL(gpis_grad_finalize, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, partial, M, M_pad,
                     n_parts, sel, var, gstd);
}

size_t gpis_v_bytes(const cdx_gpis& g, int64_t M) {
  return (size_t)round_up(M, ST_BM) * (size_t)g.N_pad * sizeof(double);
}

int gpis_var_launch(const cdx_gpis& g, const double* X, int64_t M, double* std_out, double* var_out, void* ws,
                    hipStream_t s, double* vout) {
  if (M <= 0) return CDX_OK;
  const int64_t M_pad = round_up(M, ST_BM);
  const int n_tiles = g.N_pad / ST_BN;
  if (M_pad / ST_BM * n_tiles > 0x7fffffff) return CDX_EINVAL;
  const int Mt = (int)(M_pad / ST_BM);
  double* partial = static_cast<double*>(ws);
  switch (g.kernel) {
    case CDX_KERNEL_TPS: var_launch_kt<CDX_KERNEL_TPS>(g, X, M, std_out, var_out, partial, M_pad, Mt, n_tiles, vout, s); break;
    case CDX_KERNEL_RBF: var_launch_kt<CDX_KERNEL_RBF>(g, X, M, std_out, var_out, partial, M_pad, Mt, n_tiles, vout, s); break;
    default: var_launch_kt<CDX_KERNEL_JOINT>(g, X, M, std_out, var_out, partial, M_pad, Mt, n_tiles, vout, s); break;
  }
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int gpis_grad_launch(const cdx_gpis& g, const double* X, int64_t M, const int64_t* sel, const double* var,
                     double* gstd, void* ws, hipStream_t s, const double* vin) {
  if (vin && !g.Linv) return CDX_EINVAL;
  if (M <= 0) return CDX_OK;
  const int64_t M_pad = round_up(M, ST_BM);
  const int n_tiles = g.N_pad / ST_BN;
  if (M_pad / ST_BM * (int64_t)16 * n_tiles * (n_tiles + 1) / 2 > 0x7fffffff) return CDX_EINVAL;
  const int Mt = (int)(M_pad / ST_BM);
  double* partial = static_cast<double*>(ws);
  switch (g.kernel) {
    case CDX_KERNEL_TPS: grad_launch_kt<CDX_KERNEL_TPS>(g, X, M, sel, var, gstd, partial, M_pad, Mt, n_tiles, vin, s); break;
    case CDX_KERNEL_RBF: grad_launch_kt<CDX_KERNEL_RBF>(g, X, M, sel, var, gstd, partial, M_pad, Mt, n_tiles, vin, s); break;
    default: grad_launch_kt<CDX_KERNEL_JOINT>(g, X, M, sel, var, gstd, partial, M_pad, Mt, n_tiles, vin, s); break;
  }
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
    case CDX_KERNEL_TPS: hipLaunchKernelGGL(gpis_mean_kernel<CDX_KERNEL_TPS>, grid, dim3(MEAN_BLOCK), 0, s, *g, X, M, mean, grad_mean, normal); break;
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

// Test hook: D[16×16] = A[16×4]·B[4×16] through one v_mfma_f64_16x16x4_f64 (layout check).
int cdx_selftest_mfma_f64(const double* A, const double* B, double* D, cdx_stream_t stream) {
  if (!A || !B || !D) return CDX_EINVAL;
  hipLaunchKernelGGL(mfma_f64_selftest_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), A, B, D);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

}  // extern "C"
