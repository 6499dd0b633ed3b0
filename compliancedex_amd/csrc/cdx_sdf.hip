// TorchSDF replacement for gfx950: brute-force point → triangle-mesh squared distance,
// sign, unit (p − c) normal and closest point, plus the argmin face index.
//
// Mapping: one point per lane, 256-point workgroups; faces are streamed through LDS in
// 512-face tiles (18 KiB) and every lane walks the tile with broadcast LDS reads.  The
// 512-face tile is also the reference's tie/NaN semantics unit (cdx_sdf.h).
#include <hip/hip_runtime.h>

#include "cdx_sdf.h"

#pragma clang fp contract(off)

namespace {

constexpr int SDF_BLOCK = 256;
constexpr int SDF_TILE = CDX_SDF_REF_TILE;

__global__ __launch_bounds__(SDF_BLOCK) void sdf_forward_kernel(const float* __restrict__ points, int64_t P,
                                                                const float* __restrict__ faces, int64_t F,
                                                                float* __restrict__ out_dist, int32_t* __restrict__ out_sign,
                                                                float* __restrict__ out_nrm, float* __restrict__ out_clst,
                                                                int32_t* __restrict__ out_face) {
  __shared__ float sf[SDF_TILE * 9];
  const int64_t pi = (int64_t)blockIdx.x * SDF_BLOCK + threadIdx.x;
  const bool live = pi < P;
  cdx::F3 p = cdx::f3(0.f, 0.f, 0.f);
  if (live) p = cdx::f3(points[3 * pi], points[3 * pi + 1], points[3 * pi + 2]);
  float best = 0.f;
  int bsign = 0, bface = -1;
  cdx::F3 bn = cdx::f3(0.f, 0.f, 0.f), bc = bn;
  for (int64_t f0 = 0; f0 < F; f0 += SDF_TILE) {
    const int nt = (int)min((int64_t)SDF_TILE, F - f0);
    __syncthreads();
    for (int j = threadIdx.x; j < nt * 9; j += SDF_BLOCK) sf[j] = faces[f0 * 9 + j];
    __syncthreads();
    float tbest = 0.f;
    int tsign = 0, tface = -1;
    cdx::F3 tn = cdx::f3(0.f, 0.f, 0.f), tc = tn;
    for (int s = 0; s < nt; ++s) {
      const float* v = &sf[9 * s];
      cdx::F3 c, n;
      int sg;
      const float d = cdx::point_face(p, cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]),
                                      cdx::f3(v[6], v[7], v[8]), c, n, sg);
      if (s == 0 || tbest > d) { tbest = d; tsign = sg; tn = n; tc = c; tface = (int)(f0 + s); }
    }
    if (f0 == 0 || best > tbest) { best = tbest; bsign = tsign; bn = tn; bc = tc; bface = tface; }
  }
  if (!live) return;
  out_dist[pi] = best;
  out_sign[pi] = bsign;
  out_nrm[3 * pi] = bn.x; out_nrm[3 * pi + 1] = bn.y; out_nrm[3 * pi + 2] = bn.z;
  out_clst[3 * pi] = bc.x; out_clst[3 * pi + 1] = bc.y; out_clst[3 * pi + 2] = bc.z;
  if (out_face) out_face[pi] = bface;
}

__global__ __launch_bounds__(256) void sdf_backward_kernel(const float* __restrict__ gd, const float* __restrict__ points,
                                                           const float* __restrict__ clst, int64_t P,
                                                           float* __restrict__ gp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const float g = 2.f * gd[i];
  for (int c = 0; c < 3; ++c) gp[3 * i + c] = (points[3 * i + c] - clst[3 * i + c]) * g;
}

}  // namespace

extern "C" {

int cdx_sdf_forward(const float* points, int64_t P, const float* faces, int64_t F, float* sqdist, int32_t* sign,
                    float* normals, float* clst, int32_t* face_idx, cdx_stream_t stream) {
  if (P < 0 || F < 0) return CDX_EINVAL;
  if (P == 0) return CDX_OK;
  if (F == 0 || !points || !faces || !sqdist || !sign || !normals || !clst) return CDX_EINVAL;
  hipLaunchKernelGGL(sdf_forward_kernel, dim3((unsigned)((P + SDF_BLOCK - 1) / SDF_BLOCK)), dim3(SDF_BLOCK), 0,
                     reinterpret_cast<hipStream_t>(stream), points, P, faces, F, sqdist, sign, normals, clst, face_idx);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_sdf_backward(const float* grad_dist, const float* points, const float* clst, int64_t P, float* grad_points,
                     cdx_stream_t stream) {
  if (P < 0) return CDX_EINVAL;
  if (P == 0) return CDX_OK;
  if (!grad_dist || !points || !clst || !grad_points) return CDX_EINVAL;
  hipLaunchKernelGGL(sdf_backward_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), grad_dist, points, clst, P, grad_points);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

}  // extern "C"
