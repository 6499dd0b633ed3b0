// TorchSDF replacement for gfx950: point → triangle-mesh squared distance, sign, unit (p − c)
// normal and closest point, plus the argmin face index — bit-identical to the reference's
// brute-force scan (unbatched_triangle_distance_cuda.cu:186-246) and to oracle/sdf_oracle.c.
//
// Culled path (meshes without NaN-capable faces, the normal case):
//   1. bbox of points ∪ vertices; 30-bit Morton keys of face centroids and of points;
//      hipCUB radix sort of both (faces once per call, points so a wave is spatially coherent).
//   2. Face records (FaceRec: every per-face quantity of point_face, computed once) in Morton
//      order, in 32-face chunks with a bounding sphere (centre, radius) and a conditioning
//      margin alpha derived from the worst face's 1/sinθ.
//   3. A workgroup = 64 sorted points × 4 waves; wave w owns chunks c ≡ w (mod 4).  Pass 1
//      takes each lane's upper bound U over chunks (every face of a chunk is at most
//      (|p−c|+r)(1+α)+β away, so the answer is ≤ U²); pass 2 evaluates a chunk only when some
//      lane's lower bound L = |p−c|(1−α) − r(1+α) − β has L ≤ 0 or L² ≤ min(U², best).  β =
//      1e-4·(|p|+|c|+r) and α ≥ 1e-4 exceed every rounding error of point_face by orders of
//      magnitude, so a skipped face's computed distance is strictly greater
//      than the winner's: it can neither win nor tie.  Faces are compared lexicographically on
//      (distance, index), which, with no NaN distances, is exactly the reference's first-
//      minimum tile rule.  The four waves' winners merge in LDS; the winner's closest point,
//      normal and sign are recomputed with point_face (deterministic, so bit-identical).
// Exact path: a mesh with a face that can produce NaN (face_may_nan) runs the brute-force
// tile-rule kernel (512-face LDS tiles); a workgroup holding a non-finite or |p| > 1e4 point
// runs the tile rule on its own wave.  The choice is made on the device (no host sync).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "cdx_sdf.h"

#pragma clang fp contract(off)

namespace {

constexpr int SDF_BLOCK = 256;
constexpr int SDF_TILE = CDX_SDF_REF_TILE;
constexpr int CHUNK = 32;           // faces per culling chunk
constexpr float PT_LIM = 1e4f;      // |p| bound of the culled path (face_may_nan's premise)

struct Sphere { float cx, cy, cz, r, alpha, cnorm, _p0, _p1; };

// Diagnostic counters (cdx_sdf_stats): [0] (point, face) pairs the culled kernel evaluated — faces a wave
// evaluates exactly (its chunk not ruled out, the face itself not ruled out for every lane) × its live lanes —, [1] pairs of the brute-force scans (exact path),
// [2] points queried.  Counted only while enabled (one atomic per wave).
// [3]: chunks the culled kernel visited (a wave fetched and bound-tested their faces), summed over waves.
__device__ unsigned long long g_sdf_stats[4];
bool g_sdf_count = false;

__device__ inline unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float fkey_inv(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ inline unsigned spread10(unsigned v) {  // 10 bits → every third bit
  v &= 1023u;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// ws layout (unsigned words): [0..2] bbox min keys, [3..5] bbox max keys, [6] may-NaN flag
__global__ void sdf_init_kernel(unsigned* ws) {
  const int t = threadIdx.x;
  if (t < 3) ws[t] = 0xFFFFFFFFu;
  else if (t < 7) ws[t] = 0u;
}

__device__ inline void bb_acc(float x, float y, float z, unsigned (&lo)[3], unsigned (&hi)[3]) {
  if (!(fabsf(x) <= PT_LIM && fabsf(y) <= PT_LIM && fabsf(z) <= PT_LIM)) return;
  const unsigned k[3] = {fkey(x), fkey(y), fkey(z)};
#pragma unroll
  for (int c = 0; c < 3; ++c) { lo[c] = min(lo[c], k[c]); hi[c] = max(hi[c], k[c]); }
}

__global__ __launch_bounds__(256) void sdf_bbox_kernel(const float* __restrict__ points, int64_t P,
                                                       const float* __restrict__ faces, int64_t F, unsigned* ws) {
  unsigned lo[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, hi[3] = {0u, 0u, 0u};
  const int64_t n = P + 3 * F;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float* v = i < P ? points + 3 * i : faces + 3 * (i - P);
    bb_acc(v[0], v[1], v[2], lo, hi);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      lo[c] = min(lo[c], (unsigned)__shfl_xor((int)lo[c], o));
      hi[c] = max(hi[c], (unsigned)__shfl_xor((int)hi[c], o));
    }
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) { atomicMin(ws + c, lo[c]); atomicMax(ws + 3 + c, hi[c]); }
  }
}

__device__ inline unsigned morton(float x, float y, float z, const unsigned* ws) {
  const float v[3] = {x, y, z};
  unsigned m = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float lo = fkey_inv(ws[c]), hi = fkey_inv(ws[3 + c]);
    const float ext = hi - lo;
    float t = ext > 0.f ? (v[c] - lo) / ext : 0.f;
    t = fminf(fmaxf(t, 0.f), 1.f);  // NaN → 0
    m |= spread10((unsigned)(t * 1023.f)) << c;
  }
  return m;
}

__global__ __launch_bounds__(256) void sdf_keys_kernel(const float* __restrict__ points, int64_t P,
                                                       const float* __restrict__ faces, int64_t F,
                                                       const unsigned* __restrict__ ws, unsigned* fkeys, int* fvals,
                                                       unsigned* pkeys, int* pvals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < F) {
    const float* v = faces + 9 * i;
    const float third = 1.f / 3.f;
    fkeys[i] = morton((v[0] + v[3] + v[6]) * third, (v[1] + v[4] + v[7]) * third, (v[2] + v[5] + v[8]) * third, ws);
    fvals[i] = (int)i;
  } else if (i < F + P) {
    const int64_t j = i - F;
    pkeys[j] = morton(points[3 * j], points[3 * j + 1], points[3 * j + 2], ws);
    pvals[j] = (int)j;
  }
}

// One thread per sorted face slot; a 32-lane half-wave builds one chunk's sphere.
// fsph[j] (the culled2 kernel's per-face test in one 16-byte read): the face's sphere centre and
// br·(1 + α + 1e-4) + 1e-4·bn, α its chunk's conditioning margin — the face-dependent part of the bound's
// threshold (sdf_culled2_kernel).
// ssph[j / SUB] the same for each SUB-face run of a chunk (its bounding sphere: centre, radius·(1 + α +
// 1e-4) + 1e-4·|centre|), tested before its faces.
#ifndef CDX_SDF_SUB
#define CDX_SDF_SUB 8
#endif
constexpr int SUB = CDX_SDF_SUB;
__global__ __launch_bounds__(256) void sdf_chunk_kernel(const float* __restrict__ faces, int64_t F,
                                                        const int* __restrict__ order, cdx::FaceRec* __restrict__ rec,
                                                        Sphere* __restrict__ sph, float4* __restrict__ fsph,
                                                        float4* __restrict__ ssph, unsigned* ws) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = j < F;
  cdx::FaceRec r;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  float kappa = 0.f;
  bool bad = false;
  if (live) {
    const int f = order[j];
    const float* v = faces + 9 * (int64_t)f;
    r = cdx::face_rec(cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]), cdx::f3(v[6], v[7], v[8]), f);
    rec[j] = r;
    bad = cdx::face_may_nan(r);
    kappa = r.kappa;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      lo[c] = fminf(fminf(v[c], v[3 + c]), v[6 + c]);
      hi[c] = fmaxf(fmaxf(v[c], v[3 + c]), v[6 + c]);
    }
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(ws + 6, 1u);
  // the SUB-face run's box first (lanes j & ~(SUB − 1) … ), then the chunk's
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int o = 1; o < SUB; o <<= 1) {
      lo[c] = fminf(lo[c], __shfl_xor(lo[c], o));
      hi[c] = fmaxf(hi[c], __shfl_xor(hi[c], o));
    }
  const float sx = 0.5f * (lo[0] + hi[0]), sy = 0.5f * (lo[1] + hi[1]), sz = 0.5f * (lo[2] + hi[2]);
  float srad = 0.f;
  if (live) {
    const cdx::F3 c = cdx::f3(sx, sy, sz);
    srad = fmaxf(fmaxf(sqrtf(cdx::dotf(cdx::sub(r.v1, c), cdx::sub(r.v1, c))),
                       sqrtf(cdx::dotf(cdx::sub(r.v2, c), cdx::sub(r.v2, c)))),
                 sqrtf(cdx::dotf(cdx::sub(r.v3, c), cdx::sub(r.v3, c))));
  }
#pragma unroll
  for (int o = 1; o < SUB; o <<= 1) srad = fmaxf(srad, __shfl_xor(srad, o));
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int o = SUB; o < CHUNK; o <<= 1) {
      lo[c] = fminf(lo[c], __shfl_xor(lo[c], o));
      hi[c] = fmaxf(hi[c], __shfl_xor(hi[c], o));
    }
  const float cx = 0.5f * (lo[0] + hi[0]), cy = 0.5f * (lo[1] + hi[1]), cz = 0.5f * (lo[2] + hi[2]);
  float rad = 0.f;
  if (live) {
    const cdx::F3 c = cdx::f3(cx, cy, cz);
    rad = fmaxf(fmaxf(sqrtf(cdx::dotf(cdx::sub(r.v1, c), cdx::sub(r.v1, c))),
                      sqrtf(cdx::dotf(cdx::sub(r.v2, c), cdx::sub(r.v2, c)))),
                sqrtf(cdx::dotf(cdx::sub(r.v3, c), cdx::sub(r.v3, c))));
  }
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) {
    rad = fmaxf(rad, __shfl_xor(rad, o));
    kappa = fmaxf(kappa, __shfl_xor(kappa, o));
  }
  {
    const float a = 1e-4f + 1e-5f * kappa;  // (the chunk's alpha, as below)
    const float alpha = a < 1.f ? a : 1.f;
    if (live) fsph[j] = make_float4(r.bx, r.by, r.bz, r.br * ((1.f + alpha) + 1e-4f) + 1e-4f * r.bn);
    else if (j < (F + CHUNK - 1) / CHUNK * CHUNK) fsph[j] = make_float4(0.f, 0.f, 0.f, 0.f);  // (never tested: nf)
    // (a run without live faces gets a NaN centre: its test then always says "needed", and nf masks its faces)
    if ((j & (SUB - 1)) == 0 && j < (F + CHUNK - 1) / CHUNK * CHUNK)
      ssph[j / SUB] = make_float4(sx, sy, sz, srad * (1.f + 1e-5f) * ((1.f + alpha) + 1e-4f) +
                                               1e-4f * sqrtf(sx * sx + sy * sy + sz * sz));
  }
  if ((j & (CHUNK - 1)) == 0 && live) {
    Sphere s;
    s.cx = cx; s.cy = cy; s.cz = cz;
    s.r = rad * (1.f + 1e-5f);
    // normal-direction error of point_face's plane projection ≲ 10ε·κ; 1e-5·κ ≈ 170ε·κ.
    // alpha ≥ 1 (or a NaN kappa) makes every lower bound ≤ 0: the chunk is always evaluated.
    const float a = 1e-4f + 1e-5f * kappa;
    s.alpha = a < 1.f ? a : 1.f;
    s.cnorm = sqrtf(cx * cx + cy * cy + cz * cz);
    s._p0 = s._p1 = 0.f;
    sph[j / CHUNK] = s;
  }
}

// Reference tile rule for one point over all faces (uniform face loads); writes outputs.
__device__ void exact_point(cdx::F3 p, const float* __restrict__ faces, int64_t F, int64_t pi, float* out_dist,
                            int32_t* out_sign, float* out_nrm, float* out_clst, int32_t* out_face, bool write) {
  float best = 0.f;
  int bsign = 0, bface = -1;
  cdx::F3 bn = cdx::f3(0.f, 0.f, 0.f), bc = bn;
  for (int64_t f0 = 0; f0 < F; f0 += SDF_TILE) {
    const int nt = (int)min((int64_t)SDF_TILE, F - f0);
    float tbest = 0.f;
    int tsign = 0, tface = -1;
    cdx::F3 tn = cdx::f3(0.f, 0.f, 0.f), tc = tn;
    for (int s = 0; s < nt; ++s) {
      const float* v = faces + 9 * (f0 + s);
      cdx::F3 c, n;
      int sg;
      const float d = cdx::point_face(p, cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]),
                                      cdx::f3(v[6], v[7], v[8]), c, n, sg);
      if (s == 0 || tbest > d) { tbest = d; tsign = sg; tn = n; tc = c; tface = (int)(f0 + s); }
    }
    if (f0 == 0 || best > tbest) { best = tbest; bsign = tsign; bn = tn; bc = tc; bface = tface; }
  }
  if (!write) return;
  out_dist[pi] = best;
  out_sign[pi] = bsign;
  out_nrm[3 * pi] = bn.x; out_nrm[3 * pi + 1] = bn.y; out_nrm[3 * pi + 2] = bn.z;
  out_clst[3 * pi] = bc.x; out_clst[3 * pi + 1] = bc.y; out_clst[3 * pi + 2] = bc.z;
  if (out_face) out_face[pi] = bface;
}

__global__ __launch_bounds__(SDF_BLOCK) void sdf_culled_kernel(
    const float* __restrict__ points, int64_t P, const int* __restrict__ porder, const float* __restrict__ faces,
    int64_t F, const cdx::FaceRec* __restrict__ rec, const Sphere* __restrict__ sph, int C,
    const unsigned* __restrict__ ws, float* __restrict__ out_dist, int32_t* __restrict__ out_sign,
    float* __restrict__ out_nrm, float* __restrict__ out_clst, int32_t* __restrict__ out_face, int count) {
  if (ws[6]) return;  // mesh has a NaN-capable face: sdf_exact_kernel does this call
#if SDF_COMPACT
  __shared__ unsigned long long s_best[4][64];  // per wave: each lane's packed (distance, face) best
  __shared__ unsigned short s_pair[4][128];     // … and its pending (lane << 5 | face) pairs
#endif
  __shared__ float s_val[4][64];
  __shared__ int s_idx[4][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t j = (int64_t)blockIdx.x * 64 + lane;
  const bool live = j < P;
  const int64_t pi = porder[live ? j : P - 1];  // dead lanes shadow a live point
  const cdx::F3 p = cdx::f3(points[3 * pi], points[3 * pi + 1], points[3 * pi + 2]);
  const bool ok = fabsf(p.x) <= PT_LIM && fabsf(p.y) <= PT_LIM && fabsf(p.z) <= PT_LIM;
  if (!__all(ok)) {  // same points in every wave: uniform over the workgroup
    if (w == 0) exact_point(p, faces, F, pi, out_dist, out_sign, out_nrm, out_clst, out_face, live);
    if (count && w == 0 && lane == 0)
      atomicAdd(&g_sdf_stats[1], (unsigned long long)F * (unsigned long long)__popcll(__ballot(live)));
    return;
  }
  const float pnorm = sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);

  // pass 1: upper bound on the answer
  float ub = INFINITY;
  for (int c = w; c < C; c += 4) {
    const Sphere s = sph[c];
    const float dx = p.x - s.cx, dy = p.y - s.cy, dz = p.z - s.cz;
    const float dist = sqrtf(dx * dx + dy * dy + dz * dz);
    const float u = (dist + s.r) * (1.f + s.alpha) + 1e-4f * (pnorm + s.cnorm + s.r);
    ub = fminf(ub, u);
  }
  s_val[w][lane] = ub;
  __syncthreads();
  ub = fminf(fminf(s_val[0][lane], s_val[1][lane]), fminf(s_val[2][lane], s_val[3][lane]));
  const float T = ub * ub;
  __syncthreads();

  // pass 2: exact distances over the chunks some lane cannot rule out
  float best = INFINITY;
  int bidx = 0x7fffffff;
  unsigned evaluated = 0;  // faces of the chunks this wave evaluated (diagnostic count)
  for (int c = w; c < C; c += 4) {
    const Sphere s = sph[c];
    const float dx = p.x - s.cx, dy = p.y - s.cy, dz = p.z - s.cz;
    const float dist = sqrtf(dx * dx + dy * dy + dz * dz);
    const float L = dist * (1.f - s.alpha) - s.r * (1.f + s.alpha) - 1e-4f * (pnorm + s.cnorm + s.r);
    const bool need = !(L > 0.f && L * L > fminf(T, best));
    if (!__any(need)) continue;
    const int f0 = c * CHUNK;
    const int nf = (int)min((int64_t)CHUNK, F - f0);
    for (int k = 0; k < nf; ++k) {
      const cdx::FaceRec& r = rec[f0 + k];
#if !defined(CDX_SDF_NO_FACEBOUND)
      // The chunk test again, on the face's own sphere (FaceRec bx..bn, the chunk's conditioning margin
      // alpha): a face every lane of the wave rules out is never evaluated — its computed distance is
      // strictly above the lane's best, so it could neither win nor tie (the argument of the chunk bound).
      {
        const float fx = p.x - r.bx, fy = p.y - r.by, fz = p.z - r.bz;
        const float fd = sqrtf(fx * fx + fy * fy + fz * fz);
        const float Lf = fd * (1.f - s.alpha) - r.br * (1.f + s.alpha) - 1e-4f * (pnorm + r.bn + r.br);
        if (!__any(!(Lf > 0.f && Lf * Lf > best))) continue;
      }
#endif
      ++evaluated;
      const float d = cdx::face_dist2(p, r);
      if (d < best || (d == best && r.idx < bidx)) { best = d; bidx = r.idx; }
    }
  }
  if (count) {
    const unsigned long long nl = __popcll(__ballot(live));
    if (lane == 0) {
      atomicAdd(&g_sdf_stats[0], (unsigned long long)evaluated * nl);
      if (w == 0) atomicAdd(&g_sdf_stats[2], nl);
    }
  }
  s_val[w][lane] = best;
  s_idx[w][lane] = bidx;
  __syncthreads();
  if (w != 0 || !live) return;
#pragma unroll
  for (int v = 1; v < 4; ++v) {
    const float d = s_val[v][lane];
    const int i = s_idx[v][lane];
    if (d < best || (d == best && i < bidx)) { best = d; bidx = i; }
  }
  const float* v = faces + 9 * (int64_t)bidx;
  cdx::F3 c, n;
  int sg;
  const float d = cdx::point_face(p, cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]),
                                  cdx::f3(v[6], v[7], v[8]), c, n, sg);
  out_dist[pi] = d;
  out_sign[pi] = sg;
  out_nrm[3 * pi] = n.x; out_nrm[3 * pi + 1] = n.y; out_nrm[3 * pi + 2] = n.z;
  out_clst[3 * pi] = c.x; out_clst[3 * pi + 1] = c.y; out_clst[3 * pi + 2] = c.z;
  if (out_face) out_face[pi] = bidx;
}

// The culled kernel, staged through LDS (default; CDX_SDF_V1 builds sdf_culled_kernel above for the A/B).
// Same bounds, same winner rule, same outputs — only where the data comes from and how the per-face tests
// are ordered differ:
//   * the chunk spheres of a block of SPH_BLK chunks sit in LDS (one cooperative load per block, instead
//     of one dependent scalar load per chunk and pass);
//   * a chunk some lane cannot rule out is fetched whole into the wave's LDS buffer with 5 vector loads per
//     lane (one round trip instead of one scalar load per face), and the next such chunk's loads are
//     issued before the current one is processed;
//   * its 32 per-face bounds are tested first, branch-free, into a bit mask against the lanes' best at the
//     chunk's start (sqrt-free: fd² against the squared threshold — the 1e-4 margins dwarf the few ulps
//     the rearrangement moves), then only the faces of the mask are evaluated.
// A skipped face is one whose bound lies above every lane's best at the time of the test, and a lane's
// best only decreases: the chunk argument of sdf_culled_kernel, unchanged.
constexpr int SPH_BLK = 512;                   // chunk spheres per LDS block (12 KB)
constexpr int REC_WORDS = sizeof(cdx::FaceRec) / 4;  // 40
static_assert(REC_WORDS * CHUNK % (64 * 4) == 0, "a chunk's records load as whole dwordx4 per lane");
constexpr int REC_V4 = REC_WORDS * CHUNK / (64 * 4);   // dwordx4 loads per lane per chunk (5)

#if defined(CDX_SDF_NO_COMPACT)
#define SDF_COMPACT 0
#else
#define SDF_COMPACT 1  // pass 2 evaluates compacted (lane, face) pairs (sdf_culled2_kernel)
#endif
#ifndef CDX_SDF_SPLIT
#define CDX_SDF_SPLIT 4
#endif
constexpr int SDF_SPLIT = CDX_SDF_SPLIT;  // workgroups per 64-point group (chunk slices; 4 since the per-slice bound pass: profiles/r04y4_*)

// (distance, face) as one unsigned 64-bit word whose order is the winner rule's: a non-negative float's
// bits order as unsigned integers, ties then go to the smaller index.
__device__ inline unsigned long long pack_best(float d, int idx) {
  return ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)idx;
}

// Workgroup (g, k) of a split launch: the 64 Morton-sorted points of group g against chunk slice k (wave w
// takes chunks c ≡ 4k + w mod 4·SPLIT), its per-point winner merged into best[pi] with a 64-bit atomic
// minimum; sdf_culled_finalize_kernel then writes the outputs.  Splitting a point group over SPLIT
// workgroups shortens its critical path — one group near no face (a point deep inside or far outside)
// otherwise holds its CU while the others idle (PMC: mean wave life ≈ 1/3 of the kernel) — and gives the
// dispatcher SPLIT× more, shorter workgroups to balance.  Each workgroup first takes the upper bound over
// its own slice's chunks (pass 1; the slices interleave over the whole Morton order, so the bound stays
// close to the one over all chunks) and the faces of the slice's chunk nearest the group's middle point
// (the seed, shared over its waves), so every slice starts with a best near the true distance; a face is still skipped only when
// its bound lies above the lane's best (which only decreases), so the global lexicographic minimum over the
// evaluated faces is the brute-force winner.  Pass 2 evaluates (lane, face) pairs, not faces: each lane keeps
// the mask of the chunk's faces its own bounds cannot rule out, and the wave packs those pairs 64 to a round
// (SDF_COMPACT; a wave of far points otherwise evaluated every face any lane needed — 3× the pairs).
// (The order of evaluation is free: the result is a minimum.)
__global__ __launch_bounds__(SDF_BLOCK) void sdf_culled2_kernel(
    const float* __restrict__ points, int64_t P, const int* __restrict__ porder, const float* __restrict__ faces,
    int64_t F, const cdx::FaceRec* __restrict__ rec, const Sphere* __restrict__ sph, int C,
    const unsigned* __restrict__ ws, float* __restrict__ out_dist, int32_t* __restrict__ out_sign,
    float* __restrict__ out_nrm, float* __restrict__ out_clst, int32_t* __restrict__ out_face,
    unsigned long long* __restrict__ best_out, const float4* __restrict__ fsph, const float4* __restrict__ ssph,
    int count) {
  if (ws[6]) return;  // mesh has a NaN-capable face: sdf_exact_kernel does this call
  __shared__ float4 s_sa[SPH_BLK];  // cx, cy, cz, r
  __shared__ float2 s_sb[SPH_BLK];  // alpha, cnorm
  __shared__ float4 s_rec[4][REC_WORDS * CHUNK / 4];  // per wave: one chunk's face records
  __shared__ float4 s_fs[4][CHUNK];                   // … and its per-face bounds (sdf_chunk_kernel fsph)
  __shared__ float4 s_ss[4][CHUNK / SUB];             // … and its SUB-face runs' bounds (ssph)
#if SDF_COMPACT
  __shared__ unsigned long long s_best[4][64];  // per wave: each lane's packed (distance, face) best
  __shared__ unsigned short s_pair[4][128];     // … and its pending (lane << 5 | face) pairs
#endif
  __shared__ float s_val[4][64];
  __shared__ int s_idx[4][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = blockIdx.x / SDF_SPLIT, slice = blockIdx.x - grp * SDF_SPLIT;
  const int64_t j = (int64_t)grp * 64 + lane;
  const bool live = j < P;
  const int64_t pi = porder[live ? j : P - 1];  // dead lanes shadow a live point
  const cdx::F3 p = cdx::f3(points[3 * pi], points[3 * pi + 1], points[3 * pi + 2]);
  const bool ok = fabsf(p.x) <= PT_LIM && fabsf(p.y) <= PT_LIM && fabsf(p.z) <= PT_LIM;
  if (!__all(ok)) {  // same points in every wave and slice: uniform over the workgroup
    if (w == 0 && slice == 0) exact_point(p, faces, F, pi, out_dist, out_sign, out_nrm, out_clst, out_face, live);
    if (count && w == 0 && slice == 0 && lane == 0)
      atomicAdd(&g_sdf_stats[1], (unsigned long long)F * (unsigned long long)__popcll(__ballot(live)));
    return;
  }
  const float pnorm = sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
  auto stage = [&](int cb) {  // spheres of chunks [cb, cb + SPH_BLK) into LDS (all waves)
    __syncthreads();
    const int nb = min(SPH_BLK, C - cb);
    for (int i = threadIdx.x; i < nb; i += SDF_BLOCK) {
      const Sphere sp = sph[cb + i];
      s_sa[i] = make_float4(sp.cx, sp.cy, sp.cz, sp.r);
      s_sb[i] = make_float2(sp.alpha, sp.cnorm);
    }
    __syncthreads();
    return nb;
  };

  // pass 1 (this slice's chunks — any subset bounds the answer from above, and the slices interleave over
  // the whole Morton order): upper bound on the answer, and the chunk that gives it (the lane's nearest,
  // roughly)
  float ub = INFINITY;
  int uc = 0;
#if defined(CDX_SDF_PASS1_ALL)
  constexpr int p1s = 4;
  const int p1c = w;
#else
  constexpr int p1s = 4 * SDF_SPLIT;
  const int p1c = 4 * slice + w;
#endif
  for (int cb = 0; cb < C; cb += SPH_BLK) {
    const int nb = stage(cb);
    for (int c = (int)(((int64_t)p1c - cb) % p1s + p1s) % p1s; c < nb; c += p1s) {
      const float4 a = s_sa[c];
      const float2 b = s_sb[c];
      const float dx = p.x - a.x, dy = p.y - a.y, dz = p.z - a.z;
      const float dist = sqrtf(dx * dx + dy * dy + dz * dz);
      const float u = (dist + a.w) * (1.f + b.x) + 1e-4f * (pnorm + b.y + a.w);
      if (u < ub) { ub = u; uc = cb + c; }
    }
  }
  s_val[w][lane] = ub;
  s_idx[w][lane] = uc;
  __syncthreads();
  int seed = s_idx[0][lane];
  {
    float m = s_val[0][lane];
#pragma unroll
    for (int v = 1; v < 4; ++v)
      if (s_val[v][lane] < m) { m = s_val[v][lane]; seed = s_idx[v][lane]; }
    ub = m;
  }
  const float T = ub * ub;
  seed = __builtin_amdgcn_readlane(seed, 32);

  // the seed chunk's faces, split over the waves (faces k ≡ w mod 4), merged in LDS: every wave of the
  // workgroup starts with the same (best, face)
  const float4* rec4 = reinterpret_cast<const float4*>(rec);
  float4* buf = s_rec[w];
  float best = INFINITY;
  int bidx = 0x7fffffff;
  unsigned evaluated = 0, visits = 0, pairs = 0;  // faces evaluated / chunks visited by this wave (diagnostic counts)
  {
    const int nf = (int)min((int64_t)CHUNK, F - (int64_t)seed * CHUNK);
    for (int k = w; k < nf; k += 4) {
      const cdx::FaceRec r = rec[(int64_t)seed * CHUNK + k];
      const float d = cdx::face_dist2(p, r);
      if (d < best || (d == best && r.idx < bidx)) { best = d; bidx = r.idx; }
      ++evaluated;
    }
    __syncthreads();  // pass 1's s_val / s_idx reads are done
    s_val[w][lane] = best;
    s_idx[w][lane] = bidx;
    __syncthreads();
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float d = s_val[v][lane];
      const int i = s_idx[v][lane];
      if (d < best || (d == best && i < bidx)) { best = d; bidx = i; }
    }
    __syncthreads();  // s_val / s_idx are written again at the end
  }
#if SDF_COMPACT
  s_best[w][lane] = pack_best(best, bidx);
#endif

  // pass 2 (this slice's chunks): exact distances over the chunks some lane cannot rule out
  const int c0 = 4 * slice + w, cs = 4 * SDF_SPLIT;
  for (int cb = 0; cb < C; cb += SPH_BLK) {
    const int nb = C <= SPH_BLK ? C : stage(cb);  // (one block: still staged from pass 1)
    // the wave's next chunk ≥ c (c ≡ c0 mod cs) some lane cannot rule out (uniform), or ≥ nb
    auto next_needed = [&](int c) {
      for (; c < nb; c += cs) {
        const float4 a = s_sa[c];
        const float2 b = s_sb[c];
        const float dx = p.x - a.x, dy = p.y - a.y, dz = p.z - a.z;
        const float dist = sqrtf(dx * dx + dy * dy + dz * dz);
        const float L = dist * (1.f - b.x) - a.w * (1.f + b.x) - 1e-4f * (pnorm + b.y + a.w);
        if (__any(!(L > 0.f && L * L > fminf(T, best)))) break;
      }
      return c;
    };
    // first chunk of the slice in this block: c ≡ c0 (mod cs), c ≥ 0 relative to cb
    const int cfirst = (int)(((int64_t)c0 - cb) % cs + cs) % cs;
    int c = next_needed(cfirst);
    float4 pre[REC_V4], pref = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < nb) {
#pragma unroll
      for (int i = 0; i < REC_V4; ++i) pre[i] = rec4[(int64_t)(cb + c) * (REC_WORDS * CHUNK / 4) + lane + 64 * i];
      if (lane < CHUNK) pref = fsph[(int64_t)(cb + c) * CHUNK + lane];
      else if (lane < CHUNK + CHUNK / SUB) pref = ssph[(int64_t)(cb + c) * (CHUNK / SUB) + lane - CHUNK];
    }
    while (c < nb) {
#pragma unroll
      for (int i = 0; i < REC_V4; ++i) buf[lane + 64 * i] = pre[i];
      if (lane < CHUNK) s_fs[w][lane] = pref;
      else if (lane < CHUNK + CHUNK / SUB) s_ss[w][lane - CHUNK] = pref;
      const int cur = c;
      const int64_t f0 = (int64_t)(cb + cur) * CHUNK;
      const float alpha = s_sb[cur].x;
      c = next_needed(cur + cs);
      if (c < nb) {  // the next chunk's records in flight while this one is processed
#pragma unroll
        for (int i = 0; i < REC_V4; ++i) pre[i] = rec4[(int64_t)(cb + c) * (REC_WORDS * CHUNK / 4) + lane + 64 * i];
        if (lane < CHUNK) pref = fsph[(int64_t)(cb + c) * CHUNK + lane];
        else if (lane < CHUNK + CHUNK / SUB) pref = ssph[(int64_t)(cb + c) * (CHUNK / SUB) + lane - CHUNK];
      }
      const cdx::FaceRec* rr = reinterpret_cast<const cdx::FaceRec*>(buf);
      const int nf = (int)min((int64_t)CHUNK, F - f0);
      ++visits;
      // per-face bounds against the lane's best: bit k set = some lane cannot rule face k out
      const float sb = sqrtf(best);  // (INF while the lane has no face yet)
      // skip ⇔ fd·(1 − α) > br·(1 + α) + β + sqrt(best), β = 1e-4·(|p| + bn + br) (the chunk bound's Lf > 0
      // ∧ Lf² > best), as th = (br·(1 + α + 1e-4) + 1e-4·bn + (1e-4·|p| + sqrt(best))) / (1 − α) with the
      // chunk's and the lane's terms hoisted and explicit FMAs: the rearrangement moves the threshold by
      // a few ulps, nothing against the 1e-4 margins (α = 1: 1/(1 − α) = ∞, never skipped)
      // (the face's part br·(1 + α + 1e-4) + 1e-4·bn comes precomputed with its centre, fsph)
      const float ia1 = 1.f / (1.f - alpha), k0 = fmaf(1e-4f, pnorm, sb);
#if defined(CDX_SDF_TH_FMA)
      const float k1 = k0 * ia1;
#endif
      unsigned mask = 0;
#if SDF_COMPACT
      unsigned lmask = 0;  // this lane's faces
#endif
      for (int sr = 0; sr < CHUNK / SUB; ++sr) {
#if !defined(CDX_SDF_NO_FACEBOUND)
        {  // the run's sphere first: a run every lane rules out skips its SUB face tests
          const float4 ss = s_ss[w][sr];
          const float ux = p.x - ss.x, uy = p.y - ss.y, uz = p.z - ss.z;
          const float ud2 = fmaf(ux, ux, fmaf(uy, uy, uz * uz));
#if defined(CDX_SDF_TH_FMA)
          const float uth = fmaf(ss.w, ia1, k1);
#else
          const float uth = (ss.w + k0) * ia1;
#endif
          if (!__any(!(ud2 > uth * uth))) continue;
        }
#endif
#pragma unroll
        for (int kk = 0; kk < SUB; ++kk) {
          const int k = SUB * sr + kk;
#if !defined(CDX_SDF_NO_FACEBOUND)
          const float4 fs = s_fs[w][k];
          const float fx = p.x - fs.x, fy = p.y - fs.y, fz = p.z - fs.z;
          const float fd2 = fmaf(fx, fx, fmaf(fy, fy, fz * fz));
#if defined(CDX_SDF_TH_FMA)
          const float th = fmaf(fs.w, ia1, k1);
#else
          const float th = (fs.w + k0) * ia1;
#endif
          const bool need = !(fd2 > th * th);
#else
          const bool need = true;
#endif
#if SDF_COMPACT
          if (need && k < nf && live) lmask |= 1u << k;
          if (__any(need && live) && k < nf) mask |= 1u << k;
#else
          if (__any(need) && k < nf) mask |= 1u << k;
#endif
        }
      }
#if SDF_COMPACT
      // the (lane, face) pairs some lane needs, packed 64 to a round: lane i of a round evaluates pair i
      // (its point read from the owning lane) and folds the result into the owner's packed best in LDS
      // with a 64-bit minimum (the same lexicographic (distance, index) order); the owners read their
      // best back after the chunk.  A face only some lanes need no longer costs the whole wave.
      auto eval_round = [&](int n) {
        const unsigned e = s_pair[w][lane];
        const int l = lane < n ? (int)(e >> 5) : lane;
        const float qx = __shfl(p.x, l), qy = __shfl(p.y, l), qz = __shfl(p.z, l);
        if (lane < n) {
          const cdx::FaceRec& r = rr[e & 31u];
          const float d = cdx::face_dist2(cdx::f3(qx, qy, qz), r);
          atomicMin(&s_best[w][l], pack_best(d, r.idx));
        }
        pairs += (unsigned)n;
      };
      int cnt = 0;
      while (mask) {
        const int k = __builtin_ctz(mask);
        mask &= mask - 1;
        const bool mine = (lmask >> k) & 1u;
        const unsigned long long b = __ballot(mine);
        if (mine)
          s_pair[w][cnt + __builtin_amdgcn_mbcnt_hi((unsigned)(b >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b, 0u))] =
              (unsigned short)((lane << 5) | k);
        cnt += __popcll(b);
        if (cnt >= 64) {
          eval_round(64);
          cnt -= 64;
          const unsigned short tail = s_pair[w][64 + lane];  // (read before any lane overwrites its slot)
          __builtin_amdgcn_wave_barrier();
          if (lane < cnt) s_pair[w][lane] = tail;
        }
      }
      if (cnt > 0) eval_round(cnt);
      {
        const unsigned long long bb = s_best[w][lane];
        best = __uint_as_float((unsigned)(bb >> 32));
        bidx = (int)(unsigned)bb;
      }
#else
      while (mask) {
        const int k = __builtin_ctz(mask);
        mask &= mask - 1;
        const cdx::FaceRec& r = rr[k];
        ++evaluated;
        const float d = cdx::face_dist2(p, r);
        if (d < best || (d == best && r.idx < bidx)) { best = d; bidx = r.idx; }
      }
#endif
    }
  }
  if (count) {
    const unsigned long long nl = __popcll(__ballot(live));
    if (lane == 0) {
      atomicAdd(&g_sdf_stats[0], (unsigned long long)evaluated * nl + pairs);
      atomicAdd(&g_sdf_stats[3], (unsigned long long)visits);
      if (w == 0 && slice == 0) atomicAdd(&g_sdf_stats[2], nl);
    }
  }
  s_val[w][lane] = best;
  s_idx[w][lane] = bidx;
  __syncthreads();
  if (w != 0 || !live) return;
#pragma unroll
  for (int v = 1; v < 4; ++v) {
    const float d = s_val[v][lane];
    const int i = s_idx[v][lane];
    if (d < best || (d == best && i < bidx)) { best = d; bidx = i; }
  }
  atomicMin(best_out + pi, pack_best(best, bidx));
}

// The outputs of the split launch's winners: point_face of each point's best face (the workgroups that ran
// the brute-force rule or a NaN-capable mesh left best at ~0 and wrote their outputs themselves).
__global__ __launch_bounds__(256) void sdf_culled_finalize_kernel(
    const float* __restrict__ points, int64_t P, const float* __restrict__ faces,
    const unsigned long long* __restrict__ best, float* __restrict__ out_dist, int32_t* __restrict__ out_sign,
    float* __restrict__ out_nrm, float* __restrict__ out_clst, int32_t* __restrict__ out_face) {
  const int64_t pi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pi >= P) return;
  const unsigned long long b = best[pi];
  if (b == ~0ull) return;
  const int bidx = (int)(unsigned)(b & 0xFFFFFFFFu);
  const cdx::F3 p = cdx::f3(points[3 * pi], points[3 * pi + 1], points[3 * pi + 2]);
  const float* v = faces + 9 * (int64_t)bidx;
  cdx::F3 cc, n;
  int sg;
  const float d = cdx::point_face(p, cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]),
                                  cdx::f3(v[6], v[7], v[8]), cc, n, sg);
  out_dist[pi] = d;
  out_sign[pi] = sg;
  out_nrm[3 * pi] = n.x; out_nrm[3 * pi + 1] = n.y; out_nrm[3 * pi + 2] = n.z;
  out_clst[3 * pi] = cc.x; out_clst[3 * pi + 1] = cc.y; out_clst[3 * pi + 2] = cc.z;
  if (out_face) out_face[pi] = bidx;
}

// Brute force with the reference's tile rule: one point per lane, faces streamed through LDS
// in 512-face tiles.  Runs when ws (if given) flags a NaN-capable face.
__global__ __launch_bounds__(SDF_BLOCK) void sdf_exact_kernel(const float* __restrict__ points, int64_t P,
                                                              const float* __restrict__ faces, int64_t F,
                                                              const unsigned* __restrict__ ws,
                                                              float* __restrict__ out_dist, int32_t* __restrict__ out_sign,
                                                              float* __restrict__ out_nrm, float* __restrict__ out_clst,
                                                              int32_t* __restrict__ out_face, int count) {
  if (ws && !ws[6]) return;
  __shared__ float sf[SDF_TILE * 9];
  const int64_t pi = (int64_t)blockIdx.x * SDF_BLOCK + threadIdx.x;
  const bool live = pi < P;
  if (count) {
    const unsigned long long nl = __popcll(__ballot(live));
    if ((threadIdx.x & 63) == 0 && nl) {
      atomicAdd(&g_sdf_stats[1], (unsigned long long)F * nl);
      atomicAdd(&g_sdf_stats[2], nl);
    }
  }
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

// Double inputs (.cu:282 dispatch): brute force with the tile rule, 512-face tiles of doubles in LDS
// (36 KB), one point per lane.  Not a hot path (the reference's live path is float32).
__global__ __launch_bounds__(SDF_BLOCK) void sdf_exact_f64_kernel(const double* __restrict__ points, int64_t P,
                                                                  const double* __restrict__ faces, int64_t F,
                                                                  double* __restrict__ out_dist,
                                                                  int32_t* __restrict__ out_sign,
                                                                  double* __restrict__ out_nrm,
                                                                  double* __restrict__ out_clst,
                                                                  int32_t* __restrict__ out_face) {
  __shared__ double sf[SDF_TILE * 9];
  const int64_t pi = (int64_t)blockIdx.x * SDF_BLOCK + threadIdx.x;
  const bool live = pi < P;
  cdx::D3 p = cdx::d3(0.0, 0.0, 0.0);
  if (live) p = cdx::d3(points[3 * pi], points[3 * pi + 1], points[3 * pi + 2]);
  double best = 0.0;
  int bsign = 0, bface = -1;
  cdx::D3 bn = cdx::d3(0.0, 0.0, 0.0), bc = bn;
  for (int64_t f0 = 0; f0 < F; f0 += SDF_TILE) {
    const int nt = (int)min((int64_t)SDF_TILE, F - f0);
    __syncthreads();
    for (int j = threadIdx.x; j < nt * 9; j += SDF_BLOCK) sf[j] = faces[f0 * 9 + j];
    __syncthreads();
    double tbest = 0.0;
    int tsign = 0, tface = -1;
    cdx::D3 tn = cdx::d3(0.0, 0.0, 0.0), tc = tn;
    for (int s = 0; s < nt; ++s) {
      const double* v = &sf[9 * s];
      cdx::D3 c, n;
      int sg;
      const double d = (double)cdx::point_face_d(p, cdx::d3(v[0], v[1], v[2]), cdx::d3(v[3], v[4], v[5]),
                                                 cdx::d3(v[6], v[7], v[8]), c, n, sg);
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

__global__ __launch_bounds__(256) void sdf_backward_f64_kernel(const double* __restrict__ gd,
                                                               const double* __restrict__ points,
                                                               const double* __restrict__ clst, int64_t P,
                                                               double* __restrict__ gp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const double g = 2. * gd[i];
  for (int c = 0; c < 3; ++c) gp[3 * i + c] = (points[3 * i + c] - clst[3 * i + c]) * g;
}

__global__ __launch_bounds__(256) void sdf_backward_kernel(const float* __restrict__ gd, const float* __restrict__ points,
                                                           const float* __restrict__ clst, int64_t P,
                                                           float* __restrict__ gp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const float g = 2.f * gd[i];
  for (int c = 0; c < 3; ++c) gp[3 * i + c] = (points[3 * i + c] - clst[3 * i + c]) * g;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int sdf_mode() {  // CDX_SDF_MODE=exact forces the brute-force kernel (benchmarks, A/B tests)
  static const int m = [] {
    const char* e = getenv("CDX_SDF_MODE");
    return (e && e[0] == 'e') ? 1 : 0;
  }();
  return m;
}

// Prepared mesh: [ws words: bbox min keys ×3, max keys ×3, may-NaN flag, 0][records: C·CHUNK FaceRec][spheres]
// [face bounds: C·CHUNK float4][run bounds: C·CHUNK/SUB float4]
size_t mesh_rec_off() { return align256(8 * sizeof(unsigned)); }
size_t mesh_sph_off(int64_t C) { return mesh_rec_off() + align256((size_t)C * CHUNK * sizeof(cdx::FaceRec)); }
size_t mesh_fsph_off(int64_t C) { return mesh_sph_off(C) + align256((size_t)C * sizeof(Sphere)); }
size_t mesh_ssph_off(int64_t C) { return mesh_fsph_off(C) + align256((size_t)C * CHUNK * sizeof(float4)); }
size_t mesh_bytes(int64_t F) {
  const int64_t C = (F + CHUNK - 1) / CHUNK;
  return mesh_ssph_off(C) + align256((size_t)C * (CHUNK / SUB) * sizeof(float4));
}

// Face records and chunk spheres in Morton order of the bounding box of the faces (and of the points,
// when given: the one-shot cdx_sdf_forward keeps its point-inclusive frame).  The order only steers the
// culling (ties resolve by face index), so any frame gives identical outputs.
int mesh_build(const float* faces, int64_t F, const float* points, int64_t P, char* mesh, hipStream_t s) {
  const int n = (int)F;
  const int C = (n + CHUNK - 1) / CHUNK;
  size_t tf = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tf, (unsigned*)nullptr, (unsigned*)nullptr, (int*)nullptr,
                                         (int*)nullptr, n, 0, 30, s) != hipSuccess)
    return CDX_ELAUNCH;
  size_t off = 0;
  const size_t o_fk = off; off = align256(off + 2 * (size_t)n * sizeof(unsigned));
  const size_t o_fv = off; off = align256(off + 2 * (size_t)n * sizeof(int));
  const size_t o_tmp = off; off = align256(off + tf);
  char* base = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&base), off, s) != hipSuccess) return CDX_ELAUNCH;
  unsigned* ws = reinterpret_cast<unsigned*>(mesh);
  unsigned* fk = reinterpret_cast<unsigned*>(base + o_fk);
  int* fv = reinterpret_cast<int*>(base + o_fv);
  hipLaunchKernelGGL(sdf_init_kernel, dim3(1), dim3(64), 0, s, ws);
  const int64_t nbb = P + 3 * F;
  const unsigned bbb = (unsigned)std::min<int64_t>((nbb + 255) / 256, 1024);
  hipLaunchKernelGGL(sdf_bbox_kernel, dim3(bbb), dim3(256), 0, s, points, P, faces, F, ws);
  hipLaunchKernelGGL(sdf_keys_kernel, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, s, (const float*)nullptr,
                     (int64_t)0, faces, F, (const unsigned*)ws, fk, fv, (unsigned*)nullptr, (int*)nullptr);
  size_t t1 = tf;
  bool ok = hipcub::DeviceRadixSort::SortPairs(base + o_tmp, t1, fk, fk + n, fv, fv + n, n, 0, 30, s) == hipSuccess;
  hipLaunchKernelGGL(sdf_chunk_kernel, dim3((unsigned)((C * CHUNK + 255) / 256)), dim3(256), 0, s, faces, F,
                     (const int*)(fv + n), reinterpret_cast<cdx::FaceRec*>(mesh + mesh_rec_off()),
                     reinterpret_cast<Sphere*>(mesh + mesh_sph_off(C)), reinterpret_cast<float4*>(mesh + mesh_fsph_off(C)),
                     reinterpret_cast<float4*>(mesh + mesh_ssph_off(C)), ws);
  ok = ok && hipGetLastError() == hipSuccess;
  ok = (hipFreeAsync(base, s) == hipSuccess) && ok;
  return ok ? CDX_OK : CDX_ELAUNCH;
}

// Points in Morton order of the mesh's frame (a wave then holds nearby points), the culled kernel, and
// the brute-force tile rule when the mesh may produce NaN distances (decided on the device).
int mesh_query(const char* mesh, const float* faces, int64_t F, const float* points, int64_t P, float* sqdist,
               int32_t* sign, float* normals, float* clst, int32_t* face_idx, hipStream_t s) {
  const int m = (int)P;
  const int C = (int)((F + CHUNK - 1) / CHUNK);
  size_t tp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tp, (unsigned*)nullptr, (unsigned*)nullptr, (int*)nullptr,
                                         (int*)nullptr, m, 0, 30, s) != hipSuccess)
    return CDX_ELAUNCH;
  size_t off = 0;
  const size_t o_pk = off; off = align256(off + 2 * (size_t)m * sizeof(unsigned));
  const size_t o_pv = off; off = align256(off + 2 * (size_t)m * sizeof(int));
  const size_t o_tmp = off; off = align256(off + tp);
  const size_t o_best = off; off = align256(off + (size_t)m * sizeof(unsigned long long));
  char* base = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&base), off, s) != hipSuccess) return CDX_ELAUNCH;
  const unsigned* ws = reinterpret_cast<const unsigned*>(mesh);
  unsigned* pk = reinterpret_cast<unsigned*>(base + o_pk);
  int* pv = reinterpret_cast<int*>(base + o_pv);
  hipLaunchKernelGGL(sdf_keys_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, points, P,
                     (const float*)nullptr, (int64_t)0, ws, (unsigned*)nullptr, (int*)nullptr, pk, pv);
  size_t t2 = tp;
  bool ok = hipcub::DeviceRadixSort::SortPairs(base + o_tmp, t2, pk, pk + m, pv, pv + m, m, 0, 30, s) == hipSuccess;
#if defined(CDX_SDF_V1)
  hipLaunchKernelGGL(sdf_culled_kernel, dim3((unsigned)((P + 63) / 64)), dim3(SDF_BLOCK), 0, s, points, P,
                     (const int*)(pv + m), faces, F, reinterpret_cast<const cdx::FaceRec*>(mesh + mesh_rec_off()),
                     reinterpret_cast<const Sphere*>(mesh + mesh_sph_off(C)), C, ws, sqdist, sign, normals, clst,
                     face_idx, (int)g_sdf_count);
#else
  unsigned long long* best = reinterpret_cast<unsigned long long*>(base + o_best);
  ok = ok && hipMemsetAsync(best, 0xFF, (size_t)m * sizeof(unsigned long long), s) == hipSuccess;
  hipLaunchKernelGGL(sdf_culled2_kernel, dim3((unsigned)((P + 63) / 64 * SDF_SPLIT)), dim3(SDF_BLOCK), 0, s, points,
                     P, (const int*)(pv + m), faces, F, reinterpret_cast<const cdx::FaceRec*>(mesh + mesh_rec_off()),
                     reinterpret_cast<const Sphere*>(mesh + mesh_sph_off(C)), C, ws, sqdist, sign, normals, clst,
                     face_idx, best, reinterpret_cast<const float4*>(mesh + mesh_fsph_off(C)),
                     reinterpret_cast<const float4*>(mesh + mesh_ssph_off(C)), (int)g_sdf_count);
  hipLaunchKernelGGL(sdf_culled_finalize_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, points, P, faces,
                     (const unsigned long long*)best, sqdist, sign, normals, clst, face_idx);
#endif
  hipLaunchKernelGGL(sdf_exact_kernel, dim3((unsigned)((P + SDF_BLOCK - 1) / SDF_BLOCK)), dim3(SDF_BLOCK), 0, s, points,
                     P, faces, F, ws, sqdist, sign, normals, clst, face_idx, (int)g_sdf_count);
  ok = ok && hipGetLastError() == hipSuccess;
  ok = (hipFreeAsync(base, s) == hipSuccess) && ok;
  return ok ? CDX_OK : CDX_ELAUNCH;
}

bool sdf_args_ok(int64_t P, const float* points, const float* faces, int64_t F, const float* sqdist,
                 const int32_t* sign, const float* normals, const float* clst) {
  return !(F == 0 || !points || !faces || !sqdist || !sign || !normals || !clst) && P <= INT32_MAX &&
         F <= INT32_MAX / 9;
}

}  // namespace

extern "C" {

int cdx_sdf_forward(const float* points, int64_t P, const float* faces, int64_t F, float* sqdist, int32_t* sign,
                    float* normals, float* clst, int32_t* face_idx, cdx_stream_t stream) {
  if (P < 0 || F < 0) return CDX_EINVAL;
  if (P == 0) return CDX_OK;
  if (!sdf_args_ok(P, points, faces, F, sqdist, sign, normals, clst)) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (sdf_mode() == 1) {
    hipLaunchKernelGGL(sdf_exact_kernel, dim3((unsigned)((P + SDF_BLOCK - 1) / SDF_BLOCK)), dim3(SDF_BLOCK), 0, s,
                       points, P, faces, F, (const unsigned*)nullptr, sqdist, sign, normals, clst, face_idx,
                       (int)g_sdf_count);
    return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
  }
  char* mesh = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&mesh), mesh_bytes(F), s) != hipSuccess) return CDX_ELAUNCH;
  int rc = mesh_build(faces, F, points, P, mesh, s);
  if (!rc) rc = mesh_query(mesh, faces, F, points, P, sqdist, sign, normals, clst, face_idx, s);
  if (hipFreeAsync(mesh, s) != hipSuccess && !rc) rc = CDX_ELAUNCH;
  return rc;
}

size_t cdx_sdf_mesh_bytes(int64_t F) { return F > 0 ? mesh_bytes(F) : 0; }

int cdx_sdf_mesh_prepare(const float* faces, int64_t F, void* mesh, cdx_stream_t stream) {
  if (F <= 0 || F > INT32_MAX / 9 || !faces || !mesh) return CDX_EINVAL;
  return mesh_build(faces, F, nullptr, 0, static_cast<char*>(mesh), reinterpret_cast<hipStream_t>(stream));
}

int cdx_sdf_query(const void* mesh, const float* faces, int64_t F, const float* points, int64_t P, float* sqdist,
                  int32_t* sign, float* normals, float* clst, int32_t* face_idx, cdx_stream_t stream) {
  if (P < 0 || F < 0 || !mesh) return CDX_EINVAL;
  if (P == 0) return CDX_OK;
  if (!sdf_args_ok(P, points, faces, F, sqdist, sign, normals, clst)) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (sdf_mode() == 1) return cdx_sdf_forward(points, P, faces, F, sqdist, sign, normals, clst, face_idx, stream);
  return mesh_query(static_cast<const char*>(mesh), faces, F, points, P, sqdist, sign, normals, clst, face_idx, s);
}

int cdx_sdf_chunk_visits(uint64_t* out, cdx_stream_t stream) {
  if (!out) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(g_sdf_stats), sizeof(uint64_t), 3 * sizeof(uint64_t),
                               hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CDX_ELAUNCH;
  return CDX_OK;
}

int cdx_sdf_stats(int32_t enable, uint64_t* out3, cdx_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (out3) {
    if (hipMemcpyFromSymbolAsync(out3, HIP_SYMBOL(g_sdf_stats), 3 * sizeof(uint64_t), 0, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return CDX_ELAUNCH;
  }
  if (enable >= 0) {
    const unsigned long long z[4] = {0, 0, 0, 0};
    if (enable && hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sdf_stats), z, sizeof(z), 0, hipMemcpyHostToDevice, s) != hipSuccess)
      return CDX_ELAUNCH;
    if (enable && hipStreamSynchronize(s) != hipSuccess) return CDX_ELAUNCH;
    g_sdf_count = enable != 0;
  }
  return CDX_OK;
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

int cdx_sdf_forward_f64(const double* points, int64_t P, const double* faces, int64_t F, double* sqdist,
                        int32_t* sign, double* normals, double* clst, int32_t* face_idx, cdx_stream_t stream) {
  if (P < 0 || F < 0) return CDX_EINVAL;
  if (P == 0) return CDX_OK;
  if (F == 0 || !points || !faces || !sqdist || !sign || !normals || !clst) return CDX_EINVAL;
  if (P > INT32_MAX || F > INT32_MAX / 9) return CDX_EINVAL;
  hipLaunchKernelGGL(sdf_exact_f64_kernel, dim3((unsigned)((P + SDF_BLOCK - 1) / SDF_BLOCK)), dim3(SDF_BLOCK), 0,
                     reinterpret_cast<hipStream_t>(stream), points, P, faces, F, sqdist, sign, normals, clst, face_idx);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_sdf_backward_f64(const double* grad_dist, const double* points, const double* clst, int64_t P,
                         double* grad_points, cdx_stream_t stream) {
  if (P < 0) return CDX_EINVAL;
  if (P == 0) return CDX_OK;
  if (!grad_dist || !points || !clst || !grad_points) return CDX_EINVAL;
  hipLaunchKernelGGL(sdf_backward_f64_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), grad_dist, points, clst, P, grad_points);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

}  // extern "C"
