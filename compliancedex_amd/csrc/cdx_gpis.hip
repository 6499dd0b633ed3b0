// GPIS query kernels for gfx950.
//
//   gpis_mean_kernel   mean = Σ α_j k(x, x_j) + bias and ∇mean (VALU, fp64); optional
//                      normal = ∇mean/(‖∇mean‖+1e-8)   — gpis.py:43-55 (mean), :63-87 (normal)
//   gpis_std_kernel    W = K*·E11⁻¹ on fp64 MFMA (v_mfma_f64_16x16x4_f64) with the K* tile
//                      generated on chip, fused epilogue reducing s = Σ_n W_mn k_mn and
//                      g = Σ_n W_mn kd_mn (x_m − x_n) per query → partial sums per
//                      column tile                                   — gpis.py:56-59
//   gpis_std_finalize  std = sqrt|k0 − s|, ∇std = −sign·g/std
//
// The reference builds the full M×M posterior covariance to read its diagonal and
// re-solves E11 on every call; here E11⁻¹ and α are precomputed once per object and
// only the diagonal is formed.
#include <hip/hip_runtime.h>

#include "cdx_gpis.h"
#include "cdx_prof.h"

using cdx::gpis_k;
using cdx::gpis_k0;

typedef double dbl4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int MEAN_BLOCK = 64;

template <int KT>
__global__ __launch_bounds__(MEAN_BLOCK) void gpis_mean_kernel(cdx_gpis g, const double* __restrict__ X, int64_t M,
                                                               double* __restrict__ mean, double* __restrict__ gmean,
                                                               double* __restrict__ normal) {
  __shared__ double sx[MEAN_BLOCK], sy[MEAN_BLOCK], sz[MEAN_BLOCK], sa[MEAN_BLOCK];
  const int64_t m = (int64_t)blockIdx.x * MEAN_BLOCK + threadIdx.x;
  double x0 = 0, x1 = 0, x2 = 0;
  if (m < M) { x0 = X[3 * m]; x1 = X[3 * m + 1]; x2 = X[3 * m + 2]; }
  const double R = g.R, inv_s2 = 1.0 / (g.sigma * g.sigma);
  double acc = 0, g0 = 0, g1 = 0, g2 = 0;
  for (int j0 = 0; j0 < g.N; j0 += MEAN_BLOCK) {
    const int j = j0 + threadIdx.x;
    __syncthreads();
    if (j < g.N) {
      sx[threadIdx.x] = g.X1[3 * j];
      sy[threadIdx.x] = g.X1[3 * j + 1];
      sz[threadIdx.x] = g.X1[3 * j + 2];
      sa[threadIdx.x] = g.alpha[j];
    }
    __syncthreads();
    const int cnt = min(MEAN_BLOCK, g.N - j0);
    for (int jj = 0; jj < cnt; ++jj) {
      const double dx = x0 - sx[jj], dy = x1 - sy[jj], dz = x2 - sz[jj];
      double k, kd;
      gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, k, kd);
      const double a = sa[jj];
      acc += a * k;
      const double ak = a * kd;
      g0 += ak * dx;
      g1 += ak * dy;
      g2 += ak * dz;
    }
  }
  if (m >= M) return;
  mean[m] = acc + g.bias;
  if (gmean) { gmean[3 * m] = g0; gmean[3 * m + 1] = g1; gmean[3 * m + 2] = g2; }
  if (normal) {
    const double nn = sqrt(g0 * g0 + g1 * g1 + g2 * g2) + 1e-8;
    normal[3 * m] = g0 / nn; normal[3 * m + 1] = g1 / nn; normal[3 * m + 2] = g2 / nn;
  }
}

// ------------------------------------------------------------------ std (MFMA)
// Tile: 64 queries × 64 output columns per 256-thread workgroup, K-step 16.
// Wave w owns rows 32·(w>>1)…+32 and columns 32·(w&1)…+32 as 2×2 MFMA 16×16 tiles.
// v_mfma_f64_16x16x4_f64 operand maps (cdna_hip_programming.md §3):
//   A: lane l holds A[row l&15][k l>>4];  B: B[k l>>4][col l&15]
//   C/D: reg r of lane l is D[row (l>>4) + 4r][col l&15]
constexpr int ST_BM = 64, ST_BN = 64, ST_BK = 16, ST_LD = 80;  // LD padded: conflict-free b64 reads

template <int KT>
__global__ __launch_bounds__(256) void gpis_std_kernel(cdx_gpis g, const double* __restrict__ X, int64_t M,
                                                       double* __restrict__ partial, int64_t M_pad) {
  __shared__ double Kt[ST_BK][ST_LD];  // K* tile, [k][m]
  __shared__ double As[ST_BK][ST_LD];  // E11⁻¹ tile, [k][n]
  __shared__ double xq[ST_BM][3];
  __shared__ double red[2][ST_BM][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * ST_BM;
  const int n0 = blockIdx.y * ST_BN;
  const int Np = g.N_pad;
  const double R = g.R, inv_s2 = 1.0 / (g.sigma * g.sigma);
  if (tid < ST_BM) {
    const int64_t m = min(m0 + tid, M - 1);  // pad rows replicate a valid query
    xq[tid][0] = X[3 * m]; xq[tid][1] = X[3 * m + 1]; xq[tid][2] = X[3 * m + 2];
  }
  __syncthreads();
  const int gm = tid & 63, gk = (tid >> 6) * 4;  // generation: this thread's query row and k sub-block
  const double qx = xq[gm][0], qy = xq[gm][1], qz = xq[gm][2];
  const int ar = tid >> 4, ac = (tid & 15) * 4;  // A-tile load: row, 4 columns
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  dbl4 acc00 = {0, 0, 0, 0}, acc01 = acc00, acc10 = acc00, acc11 = acc00;

  for (int kb = 0; kb < Np; kb += ST_BK) {
    const double2* src = reinterpret_cast<const double2*>(g.Ainv + (int64_t)(kb + ar) * Np + n0 + ac);
    const double2 v0 = src[0], v1 = src[1];
    double kv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = kb + gk + i;
      const double dx = qx - g.X1[3 * j], dy = qy - g.X1[3 * j + 1], dz = qz - g.X1[3 * j + 2];
      double kd;
      gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, kv[i], kd);
    }
    __syncthreads();
    As[ar][ac] = v0.x; As[ar][ac + 1] = v0.y; As[ar][ac + 2] = v1.x; As[ar][ac + 3] = v1.y;
#pragma unroll
    for (int i = 0; i < 4; ++i) Kt[gk + i][gm] = kv[i];
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < ST_BK; kk += 4) {
      const int kr = kk + (lane >> 4);
      const double a0 = Kt[kr][wr + (lane & 15)], a1 = Kt[kr][wr + 16 + (lane & 15)];
      const double b0 = As[kr][wc + (lane & 15)], b1 = As[kr][wc + 16 + (lane & 15)];
      acc00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc11, 0, 0, 0);
    }
  }

  // Epilogue: per owned row, s = Σ W k and g = Σ W kd (x_m − x_n) over this wave's 32 columns.
  double ps[2][4][4];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int r = 0; r < 4; ++r) ps[ti][r][0] = ps[ti][r][1] = ps[ti][r][2] = ps[ti][r][3] = 0.0;
#pragma unroll
  for (int tj = 0; tj < 2; ++tj) {
    const int n = n0 + wc + tj * 16 + (lane & 15);
    const double nx = g.X1[3 * n], ny = g.X1[3 * n + 1], nz = g.X1[3 * n + 2];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
      const dbl4 a = ti == 0 ? (tj == 0 ? acc00 : acc01) : (tj == 0 ? acc10 : acc11);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr + ti * 16 + (lane >> 4) + 4 * r;
        const double dx = xq[row][0] - nx, dy = xq[row][1] - ny, dz = xq[row][2] - nz;
        double k, kd;
        gpis_k<KT>(dx * dx + dy * dy + dz * dz, R, inv_s2, k, kd);
        const double w = a[r];
        const double wkd = w * kd;
        ps[ti][r][0] += w * k;
        ps[ti][r][1] += wkd * dx;
        ps[ti][r][2] += wkd * dy;
        ps[ti][r][3] += wkd * dz;
      }
    }
  }
  // reduce over the 16 lanes sharing (lane>>4)
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        double v = ps[ti][r][c];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        ps[ti][r][c] = v;
      }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr + ti * 16 + (lane >> 4) + 4 * r;
#pragma unroll
        for (int c = 0; c < 4; ++c) red[wave & 1][row][c] = ps[ti][r][c];
      }
  }
  __syncthreads();
  {
    const int row = tid >> 2, c = tid & 3;  // 64 rows × 4 values = 256 threads
    partial[((int64_t)blockIdx.y * M_pad + m0 + row) * 4 + c] = red[0][row][c] + red[1][row][c];
  }
}

template <int KT>
__global__ __launch_bounds__(256) void gpis_std_finalize(cdx_gpis g, const double* __restrict__ partial, int64_t M,
                                                         int64_t M_pad, int n_tiles, double* __restrict__ std_out,
                                                         double* __restrict__ gstd) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  double s = 0, g0 = 0, g1 = 0, g2 = 0;
  for (int t = 0; t < n_tiles; ++t) {
    const double* p = partial + ((int64_t)t * M_pad + m) * 4;
    s += p[0]; g0 += p[1]; g1 += p[2]; g2 += p[3];
  }
  const double v = gpis_k0<KT>(g.R) - s;
  const double sd = sqrt(fabs(v));
  std_out[m] = sd;
  if (gstd) {
    const double sg = v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0);
    const double f = -sg / sd;
    gstd[3 * m] = f * g0; gstd[3 * m + 1] = f * g1; gstd[3 * m + 2] = f * g2;
  }
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
  return g && g->X1 && g->alpha && g->N > 0 && g->N_pad >= g->N && g->N_pad % 64 == 0 && g->kernel >= 0 &&
         g->kernel <= 2;
}

int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

}  // namespace

extern "C" {

int cdx_gpis_mean(const cdx_gpis* g, const double* X, int64_t M, double* mean, double* grad_mean, double* normal,
                  cdx_stream_t stream) {
  if (!gpis_ok(g)) return g && (g->kernel < 0 || g->kernel > 2) ? CDX_EKERNEL : CDX_EINVAL;
  if (M < 0 || (M > 0 && (!X || !mean))) return CDX_EINVAL;
  if (M == 0) return CDX_OK;
  const dim3 grid((unsigned)((M + MEAN_BLOCK - 1) / MEAN_BLOCK));
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
  return (size_t)(g->N_pad / ST_BN) * (size_t)round_up(M, ST_BM) * 4 * sizeof(double);
}

int cdx_gpis_std(const cdx_gpis* g, const double* X, int64_t M, double* std_out, double* grad_std, void* workspace,
                 cdx_stream_t stream) {
  if (!gpis_ok(g) || !g->Ainv) return g && (g->kernel < 0 || g->kernel > 2) ? CDX_EKERNEL : CDX_EINVAL;
  if (M < 0 || (M > 0 && (!X || !std_out || !workspace))) return CDX_EINVAL;
  if (M == 0) return CDX_OK;
  const int64_t M_pad = round_up(M, ST_BM);
  const int n_tiles = g->N_pad / ST_BN;
  if (M_pad / ST_BM > 0x7fffffff) return CDX_EINVAL;
  double* partial = static_cast<double*>(workspace);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)(M_pad / ST_BM), (unsigned)n_tiles);
  const dim3 fgrid((unsigned)((M + 255) / 256));
  switch (g->kernel) {
    case CDX_KERNEL_TPS:
      cdx::prof_mark(cdx::PROF_GPIS_STD, true, s);
      hipLaunchKernelGGL(gpis_std_kernel<CDX_KERNEL_TPS>, grid, dim3(256), 0, s, *g, X, M, partial, M_pad);
      cdx::prof_mark(cdx::PROF_GPIS_STD, false, s);
      hipLaunchKernelGGL(gpis_std_finalize<CDX_KERNEL_TPS>, fgrid, dim3(256), 0, s, *g, partial, M, M_pad, n_tiles, std_out, grad_std);
      break;
    case CDX_KERNEL_RBF:
      cdx::prof_mark(cdx::PROF_GPIS_STD, true, s);
      hipLaunchKernelGGL(gpis_std_kernel<CDX_KERNEL_RBF>, grid, dim3(256), 0, s, *g, X, M, partial, M_pad);
      cdx::prof_mark(cdx::PROF_GPIS_STD, false, s);
      hipLaunchKernelGGL(gpis_std_finalize<CDX_KERNEL_RBF>, fgrid, dim3(256), 0, s, *g, partial, M, M_pad, n_tiles, std_out, grad_std);
      break;
    default:
      cdx::prof_mark(cdx::PROF_GPIS_STD, true, s);
      hipLaunchKernelGGL(gpis_std_kernel<CDX_KERNEL_JOINT>, grid, dim3(256), 0, s, *g, X, M, partial, M_pad);
      cdx::prof_mark(cdx::PROF_GPIS_STD, false, s);
      hipLaunchKernelGGL(gpis_std_finalize<CDX_KERNEL_JOINT>, fgrid, dim3(256), 0, s, *g, partial, M, M_pad, n_tiles, std_out, grad_std);
      break;
  }
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

// Test hook: D[16×16] = A[16×4]·B[4×16] through one v_mfma_f64_16x16x4_f64 (layout check).
int cdx_selftest_mfma_f64(const double* A, const double* B, double* D, cdx_stream_t stream) {
  if (!A || !B || !D) return CDX_EINVAL;
  hipLaunchKernelGGL(mfma_f64_selftest_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), A, B, D);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

}  // extern "C"
