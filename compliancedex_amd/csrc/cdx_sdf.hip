// TorchSDF replacement for gfx950: point → triangle-mesh squared distance, sign, unit (p − c)
// normal and closest point, plus the argmin face index — bit-identical to the reference's
// brute-force scan (unbatched_triangle_distance_cuda.cu:186-246) and to oracle/sdf_oracle.c.
//
// Culled path (meshes without NaN-capable faces, the normal case), round 5:
//   * a mesh is a three-level hierarchy over its faces in a spatially compact order: 8-face runs, 32-face
//     chunks (4 runs), 16 chunks to a top node.  Prepared meshes (cdx_sdf_mesh_prepare, queried every
//     iteration by the SDF/Kin optimisers) take the order of a median-split k-d tree on the face
//     centroids, built on the host once (chunk radius 5.3 mm median on the 16 384-face banana, against
//     10.5 mm for the round-4 Morton chunks — tools/sdf_cull_sim.py); the one-shot cdx_sdf_forward
//     sorts the centroids by Morton code in a cubic frame on the device (no host round trip).
//   * every node carries a bounding cylinder (axis = the area-weighted mean normal, centre, half-
//     thickness, radius) intersected with a bounding ball; every face a disk slab (centroid, unit
//     normal, in-plane radius, half-thickness).  Their distances are lower bounds on the distance to
//     every face inside; the slab bound leaves 10× fewer (point, face) pairs than a per-face ball
//     (tools/sdf_bound_study.py).  Node and slab data are computed in double from the f32 vertices and
//     rounded outward.
//   * one wave per 64 points (Morton-sorted in the points' own cubic frame): each lane first descends
//     greedily (nearest top node → nearest chunk → face of smallest slab bound) and evaluates that one
//     face, which gives it a near-final best; the top nodes some lane cannot rule out against those seeds
//     are tested once per workgroup (waves split them, an LDS mask); then each wave walks those top nodes
//     and the chunks some lane cannot rule out, tests the chunk's run nodes and, inside the runs some lane
//     needs, the faces' slab bounds per lane, and evaluates only the (lane, face) pairs a lane needs,
//     packed 64 to a round (ballot/mbcnt into LDS, an LDS 64-bit minimum on (distance bits, face index)
//     into the owner's best).  Runs and the shared top mask: config-4 forward 0.71 → 0.61 ms (points
//     around the mesh) and 0.775 → 0.725 ms (far), CDX_SDF_NO_RUNS / CDX_SDF_NO_TMASK build the A/B
//     (profiles/r05l_sdf_runs_tmask_ab.jsonl).
// A skip needs bound·(1 − α) − β > sqrt(best): α = 1e-4 + 1e-5·κ (κ = the worst face's 1/sinθ in the
// node; α ≥ 1 or a NaN κ never skips) and β = (1e-4 + 1e-8·κ)·(|p| + |c| + 3R) exceed every rounding error
// of point_face and of the bound (tests/test_sdf_bounds_cpu.py), so a skipped face's computed
// distance is strictly greater than the winner's: it can neither win nor tie.  Faces are compared
// lexicographically on (distance, index) — with no NaN distances, exactly the reference's first-minimum
// tile rule — and the winner's outputs are recomputed with point_face (bit-identical).
// Exact path: a mesh with a face that can produce NaN (face_may_nan) runs the brute-force tile-rule
// kernel (512-face LDS tiles); a wave holding a non-finite or |p| > 1e4 point runs the tile rule itself.
// The choice is made on the device (no host sync).
#include <hip/hip_runtime.h>

#include "cdx_ab.h"
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "cdx_sdf.h"

#pragma clang fp contract(off)

namespace {

constexpr int SDF_BLOCK = 256;
constexpr int SDF_TILE = CDX_SDF_REF_TILE;
constexpr int CHUNK = 32;           // faces per chunk (leaf node)
constexpr int TOPB = 16;            // chunks per top node
constexpr int RUN = 8;              // faces per run (a chunk's sub-group with its own node)
constexpr int RPC = 32 / RUN;       // runs per chunk
constexpr float PT_LIM = 1e4f;      // |p| bound of the culled path (face_may_nan's premise)

// Bounding volume of a node: a = (centre xyz, ball radius R), b = (cylinder axis xyz, half-thickness t),
// m = (cylinder radius rc, 1/(1 − α), w = γ·(|centre| + 3R)/(1 − α), γ) with γ = 1e-4 + 1e-8·κ.
struct Node { float4 a, b, m; };
// Disk slab of a face: a = (centroid xyz, in-plane radius r), b = (unit normal xyz, half-thickness t).
struct Slab { float4 a, b; };

// Diagnostic counters (cdx_sdf_stats): [0] (point, face) pairs the culled kernel evaluated (the greedy seed
// face of every lane plus the compacted pairs), [1] pairs of the brute-force scans (exact path), [2] points
// queried, [3] chunks the culled kernel's waves visited (tested face by face).  Counted only while enabled
// (one atomic per wave).
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

// frame words: [0..2] bbox min keys, [3..5] bbox max keys (mesh header: [6] may-NaN flag, [7] unused)
__global__ void sdf_init_kernel(unsigned* ws) {
  const int t = threadIdx.x;
  if (t < 3) ws[t] = 0xFFFFFFFFu;
  else if (t < 8) ws[t] = 0u;
}

__device__ inline void bb_acc(float x, float y, float z, unsigned (&lo)[3], unsigned (&hi)[3]) {
  if (!(fabsf(x) <= PT_LIM && fabsf(y) <= PT_LIM && fabsf(z) <= PT_LIM)) return;
  const unsigned k[3] = {fkey(x), fkey(y), fkey(z)};
#pragma unroll
  for (int c = 0; c < 3; ++c) { lo[c] = min(lo[c], k[c]); hi[c] = max(hi[c], k[c]); }
}

// Bounding box of n points (3 floats each): block b writes its partial (min keys ×3, max keys ×3) to part[6b ..]
// (no atomics: ≤ BBOX_BLOCKS partials, reduced by the keys kernel).  Block 0 also clears the mesh header's
// may-NaN flag when `flag` is given (a build's face kernel ORs into it afterwards).
constexpr int BBOX_BLOCKS = 32;
__global__ __launch_bounds__(256) void sdf_bbox_kernel(const float* __restrict__ v, int64_t n, unsigned* __restrict__ part,
                                                       unsigned* flag) {
  __shared__ unsigned s_lo[4][3], s_hi[4][3];
  unsigned lo[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, hi[3] = {0u, 0u, 0u};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bb_acc(v[3 * i], v[3 * i + 1], v[3 * i + 2], lo, hi);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      lo[c] = min(lo[c], (unsigned)__shfl_xor((int)lo[c], o));
      hi[c] = max(hi[c], (unsigned)__shfl_xor((int)hi[c], o));
    }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int c = 0; c < 3; ++c) { s_lo[w][c] = lo[c]; s_hi[w][c] = hi[c]; }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int c = threadIdx.x;
    part[6 * blockIdx.x + c] = min(min(s_lo[0][c], s_lo[1][c]), min(s_lo[2][c], s_lo[3][c]));
    part[6 * blockIdx.x + 3 + c] = max(max(s_hi[0][c], s_hi[1][c]), max(s_hi[2][c], s_hi[3][c]));
  }
  if (flag && blockIdx.x == 0 && threadIdx.x == 0) *flag = 0u;
}

// Morton code of MB bits per axis in the frame's CUBIC box (the largest extent on every axis: cells are cubes, so
// a run of codes is compact in space whatever the box's aspect).  fr: min keys ×3, max keys ×3.
__device__ inline unsigned morton(float x, float y, float z, const unsigned* fr, int mb) {
  const float lo[3] = {fkey_inv(fr[0]), fkey_inv(fr[1]), fkey_inv(fr[2])};
  const float ext = fmaxf(fmaxf(fkey_inv(fr[3]) - lo[0], fkey_inv(fr[4]) - lo[1]), fkey_inv(fr[5]) - lo[2]);
  const float v[3] = {x, y, z};
  unsigned m = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float t = ext > 0.f ? (v[c] - lo[c]) / ext : 0.f;
    t = fminf(fmaxf(t, 0.f), 1.f);  // NaN → 0
    m |= spread10((unsigned)(t * 1023.f)) << c;
  }
  return m >> (3 * (10 - mb));
}

// Morton keys (mb bits per axis) of points (centroid = false) or of face centroids (centroid = true, 9 floats a
// face), in the frame of the nb bbox partials.
__global__ __launch_bounds__(256) void sdf_keys_kernel(const float* __restrict__ v, int64_t n, int centroid,
                                                       const unsigned* __restrict__ part, int nb, int mb,
                                                       unsigned* keys, int* vals) {
  __shared__ unsigned fr[6];
  if (threadIdx.x < 6) {
    const int c = threadIdx.x;
    unsigned r = c < 3 ? 0xFFFFFFFFu : 0u;
    for (int b = 0; b < nb; ++b) r = c < 3 ? min(r, part[6 * b + c]) : max(r, part[6 * b + c]);
    fr[c] = r;
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x, y, z;
  if (centroid) {
    const float* f = v + 9 * i;
    const float third = 1.f / 3.f;
    x = (f[0] + f[3] + f[6]) * third; y = (f[1] + f[4] + f[7]) * third; z = (f[2] + f[5] + f[8]) * third;
  } else {
    x = v[3 * i]; y = v[3 * i + 1]; z = v[3 * i + 2];
  }
  keys[i] = morton(x, y, z, fr, mb);
  vals[i] = (int)i;
}

// One thread per slot j of the face order (C·CHUNK slots, the tail past F zeroed): the face record of
// point_face (FaceRec) and its disk slab, in double from the f32 vertices: centroid c (→ f32), unit normal
// n (→ f32), then relative to those rounded values the half-thickness t = max |n̂·(v − c)| and the in-plane
// radius r = max |(v − c) − (n̂·(v − c))·n̂| (n̂ = the f32 normal renormalised in double), rounded up.
// A face without a finite normal gets a NaN slab (never skipped; its mesh takes the exact path anyway).
__global__ __launch_bounds__(256) void sdf_face_kernel(const float* __restrict__ faces, int64_t F, int64_t slots,
                                                       const int* __restrict__ order, cdx::FaceRec* __restrict__ rec,
                                                       Slab* __restrict__ slab, unsigned* ws) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= slots) return;
  bool bad = false;
  if (j < F) {
    const int f = order[j];
    const float* v = faces + 9 * (int64_t)f;
    const cdx::FaceRec r = cdx::face_rec(cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]), cdx::f3(v[6], v[7], v[8]), f);
    rec[j] = r;
    bad = cdx::face_may_nan(r);
    double p[3][3];
    for (int k = 0; k < 3; ++k)
      for (int c = 0; c < 3; ++c) p[k][c] = (double)v[3 * k + c];
    double cen[3], e1[3], e2[3];
    for (int c = 0; c < 3; ++c) {
      cen[c] = (p[0][c] + p[1][c] + p[2][c]) / 3.0;
      e1[c] = p[1][c] - p[0][c];
      e2[c] = p[2][c] - p[0][c];
    }
    const double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    const double nl = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    Slab s;
    if (nl > 0.0 && nl < INFINITY) {
      const float c32[3] = {(float)cen[0], (float)cen[1], (float)cen[2]};
      const float n32[3] = {(float)(n[0] / nl), (float)(n[1] / nl), (float)(n[2] / nl)};
      const double m = sqrt((double)n32[0] * n32[0] + (double)n32[1] * n32[1] + (double)n32[2] * n32[2]);
      const double nh[3] = {n32[0] / m, n32[1] / m, n32[2] / m};
      double t = 0.0, r2 = 0.0;
      for (int k = 0; k < 3; ++k) {
        const double d[3] = {p[k][0] - c32[0], p[k][1] - c32[1], p[k][2] - c32[2]};
        const double h = d[0] * nh[0] + d[1] * nh[1] + d[2] * nh[2];
        const double e[3] = {d[0] - h * nh[0], d[1] - h * nh[1], d[2] - h * nh[2]};
        t = fmax(t, fabs(h));
        r2 = fmax(r2, e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
      }
      s.a = make_float4(c32[0], c32[1], c32[2], (float)(sqrt(r2) * (1.0 + 1e-6)));
      s.b = make_float4(n32[0], n32[1], n32[2], (float)(t * (1.0 + 1e-6)));
    } else {
      s.a = make_float4(NAN, NAN, NAN, NAN);
      s.b = make_float4(NAN, NAN, NAN, NAN);
    }
    slab[j] = s;
  } else {
    cdx::FaceRec r = {};
    r.idx = 0x7fffffff;
    rec[j] = r;
    Slab s;
    s.a = make_float4(0.f, 0.f, 0.f, 0.f);
    s.b = make_float4(0.f, 0.f, 0.f, 0.f);
    slab[j] = s;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(ws + 6, 1u);
}

__device__ inline double wave_min(double v) {
  for (int o = 32; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}
__device__ inline double wave_max(double v) {
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ inline double wave_sum(double v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One wave per node of S consecutive face slots: the node's bounding ball and cylinder, in double from the
// f32 vertices of its face records and relative to the f32-rounded centre and axis the kernel will use:
//   pass 1  box centre c, area-weighted normal sum → axis a (z if it vanishes), the faces' worst κ;
//   pass 2  extent along a → the cylinder's mid-plane, moved into the centre c;
//   pass 3  half-thickness t, cylinder radius rc, ball radius R (all rounded up by 1e-6).
// Margins: α = 1e-4 + 1e-5·κ (1 for a NaN κ: never skipped), ia1 = 1/(1 − α), γ = 1e-4 + 1e-8·κ,
// w = γ·(|c| + 3R)·ia1 (tests/test_sdf_bounds_cpu.py: point_face's absolute error stays below 1e-9·κ·(|p| + |c| + r)
// on slivers up to κ ~ 1e6, 1.4e-6·(|p| + |c| + r) on ordinary faces).
__global__ __launch_bounds__(64) void sdf_node_kernel(const cdx::FaceRec* __restrict__ rec, int64_t F, int S,
                                                      Node* __restrict__ out) {
  const int64_t f0 = (int64_t)blockIdx.x * S, f1 = min(F, f0 + S);
  const int lane = threadIdx.x;
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, ns[3] = {0, 0, 0};
  double kmax = 0.0;
  for (int64_t f = f0 + lane; f < f1; f += 64) {
    const cdx::FaceRec& r = rec[f];
    const double v[3][3] = {{r.v1.x, r.v1.y, r.v1.z}, {r.v2.x, r.v2.y, r.v2.z}, {r.v3.x, r.v3.y, r.v3.z}};
    for (int k = 0; k < 3; ++k)
      for (int c = 0; c < 3; ++c) { lo[c] = fmin(lo[c], v[k][c]); hi[c] = fmax(hi[c], v[k][c]); }
    const double e1[3] = {v[1][0] - v[0][0], v[1][1] - v[0][1], v[1][2] - v[0][2]};
    const double e2[3] = {v[2][0] - v[0][0], v[2][1] - v[0][1], v[2][2] - v[0][2]};
    ns[0] += e1[1] * e2[2] - e1[2] * e2[1];
    ns[1] += e1[2] * e2[0] - e1[0] * e2[2];
    ns[2] += e1[0] * e2[1] - e1[1] * e2[0];
    kmax = (r.kappa <= 1e30f) ? fmax(kmax, (double)r.kappa) : INFINITY;  // NaN / inf κ: never skip
  }
  double c[3], a[3];
  for (int k = 0; k < 3; ++k) {
    lo[k] = wave_min(lo[k]);
    hi[k] = wave_max(hi[k]);
    ns[k] = wave_sum(ns[k]);
    c[k] = (double)(float)(0.5 * (lo[k] + hi[k]));
  }
  kmax = wave_max(kmax);
  const double nl = sqrt(ns[0] * ns[0] + ns[1] * ns[1] + ns[2] * ns[2]);
  float a32[3] = {0.f, 0.f, 1.f};
  if (nl > 0.0 && nl < INFINITY)
    for (int k = 0; k < 3; ++k) a32[k] = (float)(ns[k] / nl);
  const double am = sqrt((double)a32[0] * a32[0] + (double)a32[1] * a32[1] + (double)a32[2] * a32[2]);
  for (int k = 0; k < 3; ++k) a[k] = a32[k] / am;
  // pass 2: the extent along the axis
  double hlo = INFINITY, hhi = -INFINITY;
  for (int64_t f = f0 + lane; f < f1; f += 64) {
    const cdx::FaceRec& r = rec[f];
    const cdx::F3 vv[3] = {r.v1, r.v2, r.v3};
    for (int k = 0; k < 3; ++k) {
      const double h = (vv[k].x - c[0]) * a[0] + (vv[k].y - c[1]) * a[1] + (vv[k].z - c[2]) * a[2];
      hlo = fmin(hlo, h);
      hhi = fmax(hhi, h);
    }
  }
  hlo = wave_min(hlo);
  hhi = wave_max(hhi);
  const double mid = f1 > f0 ? 0.5 * (hlo + hhi) : 0.0;
  for (int k = 0; k < 3; ++k) c[k] = (double)(float)(c[k] + mid * a[k]);
  // pass 3: half-thickness, cylinder radius, ball radius about the final centre
  double t = 0.0, rc2 = 0.0, R2 = 0.0;
  for (int64_t f = f0 + lane; f < f1; f += 64) {
    const cdx::FaceRec& r = rec[f];
    const cdx::F3 vv[3] = {r.v1, r.v2, r.v3};
    for (int k = 0; k < 3; ++k) {
      const double d[3] = {vv[k].x - c[0], vv[k].y - c[1], vv[k].z - c[2]};
      const double h = d[0] * a[0] + d[1] * a[1] + d[2] * a[2];
      const double e[3] = {d[0] - h * a[0], d[1] - h * a[1], d[2] - h * a[2]};
      t = fmax(t, fabs(h));
      rc2 = fmax(rc2, e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
      R2 = fmax(R2, d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    }
  }
  t = wave_max(t);
  rc2 = wave_max(rc2);
  R2 = wave_max(R2);
  if (lane != 0) return;
  const double R = sqrt(R2) * (1.0 + 1e-6);
  const double al = 1e-4 + 1e-5 * kmax;  // (inf for a NaN κ)
  const double ia1 = al < 1.0 ? 1.0 / (1.0 - al) : INFINITY;
  const double gam = 1e-4 + 1e-8 * kmax;
  const double cn = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
  Node nd;
  nd.a = make_float4((float)c[0], (float)c[1], (float)c[2], (float)R);
  nd.b = make_float4(a32[0], a32[1], a32[2], (float)(t * (1.0 + 1e-6)));
  nd.m = make_float4((float)(sqrt(rc2) * (1.0 + 1e-6)), (float)(ia1 * (1.0 + 1e-6)),
                     (float)(gam * (cn + 3.0 * R) * ia1 * (1.0 + 1e-6)), (float)(gam * (1.0 + 1e-6)));
  out[blockIdx.x] = nd;
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


// The reference tile rule for lane b's point with the faces split over the wave's lanes (all 64 lanes call it):
// per 512-face tile, the sequential rule `s == 0 || best > d` picks the tile's first face when its distance is NaN,
// else the first minimum over the tile's non-NaN distances — a (distance, face) minimum over the lanes' partial
// minima reproduces it; across tiles the same rule runs on the (uniform) tile results.  The winner's sign, normal and
// closest point are recomputed from the same point_face call the sequential scan kept.
__device__ void exact_point_wave(int b, cdx::F3 p0, int64_t pi, bool live0, const float* __restrict__ faces, int64_t F,
                                 float* out_dist, int32_t* out_sign, float* out_nrm, float* out_clst,
                                 int32_t* out_face) {
  const int lane = threadIdx.x & 63;
  const cdx::F3 p = cdx::f3(__shfl(p0.x, b), __shfl(p0.y, b), __shfl(p0.z, b));
  const int64_t pib = (int64_t)(((uint64_t)(uint32_t)__shfl((int)(pi >> 32), b) << 32) |
                                (uint64_t)(uint32_t)__shfl((int)(uint32_t)pi, b));
  const bool wr = __shfl((int)live0, b) != 0;
  float best = 0.f;
  int64_t bface = 0;
  for (int64_t f0 = 0; f0 < F; f0 += SDF_TILE) {
    const int nt = (int)min((int64_t)SDF_TILE, F - f0);
    float ld = 0.f;
    int ls = -1;  // this lane's first minimum over its non-NaN faces of the tile (−1: none)
    bool first_nan = false;
    for (int s = lane; s < nt; s += 64) {
      const float* v = faces + 9 * (f0 + s);
      cdx::F3 c, n;
      int sg;
      const float d = cdx::point_face(p, cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]),
                                      cdx::f3(v[6], v[7], v[8]), c, n, sg);
      if (s == 0) first_nan = d != d;
      if (d == d && (ls < 0 || d < ld)) { ld = d; ls = s; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float od = __shfl_xor(ld, o);
      const int os = __shfl_xor(ls, o);
      if (os >= 0 && (ls < 0 || od < ld || (od == ld && os < ls))) { ld = od; ls = os; }
    }
    const bool t_nan = __shfl((int)first_nan, 0) != 0;
    const float tbest = t_nan ? __builtin_nanf("") : ld;
    const int64_t tface = f0 + (t_nan ? 0 : ls);
    if (f0 == 0 || best > tbest) { best = tbest; bface = tface; }
  }
  if (lane != 0 || !wr) return;
  const float* v = faces + 9 * bface;
  cdx::F3 c, n;
  int sg;
  const float d = cdx::point_face(p, cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]), cdx::f3(v[6], v[7], v[8]),
                                  c, n, sg);
  out_dist[pib] = d;
  out_sign[pib] = sg;
  out_nrm[3 * pib] = n.x; out_nrm[3 * pib + 1] = n.y; out_nrm[3 * pib + 2] = n.z;
  out_clst[3 * pib] = c.x; out_clst[3 * pib + 1] = c.y; out_clst[3 * pib + 2] = c.z;
  if (out_face) out_face[pib] = (int32_t)bface;
}

// The bounds' square roots: v_sqrt_f32 (≤ 1 ulp, no correction sequence) — a bound's rounding is four orders
// below its margins; the distances themselves (point_face, face_dist2) keep the correctly rounded sqrtf.
__device__ __forceinline__ float bsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }

// Squared distance from p to a node's cylinder (its ball: *d2 = |p − c|² for the caller's ball test).
__device__ __forceinline__ float cyl_lb2(cdx::F3 p, float4 a, float4 b, float rc, float* d2) {
  const float dx = p.x - a.x, dy = p.y - a.y, dz = p.z - a.z;
  const float h = b.x * dx + b.y * dy + b.z * dz;
  const float ex = dx - h * b.x, ey = dy - h * b.y, ez = dz - h * b.z;
  const float rho = bsqrt(ex * ex + ey * ey + ez * ez);
  const float dh = fmaxf(fabsf(h) - b.w, 0.f), dr = fmaxf(rho - rc, 0.f);  // (fmaxf: NaN → 0, a bound of 0)
  *d2 = dx * dx + dy * dy + dz * dz;
  return dh * dh + dr * dr;
}

// The node's skip threshold th = (sqrt(best) + γ·|p|)/(1 − α) + w, sb = sqrt(best).
__device__ __forceinline__ float node_th(const Node& n, float sb, float pnorm) {
  return fmaf(n.m.w, pnorm, sb) * n.m.y + n.m.z;
}

// A lane cannot rule the node out: its distance bound is not above th.  Written so that any NaN (bounds, an
// infinite ia1 times a zero k0) keeps it.
__device__ __forceinline__ bool node_needed(cdx::F3 p, const Node& n, float sb, float pnorm) {
  float d2;
  const float l2 = cyl_lb2(p, n.a, n.b, n.m.x, &d2);
  const float th = node_th(n, sb, pnorm);
  const float ts = th + n.a.w;
  return !(l2 > th * th || d2 > ts * ts);
}

// Distance bound of a node for the greedy descent (larger of the cylinder's and the ball's).
__device__ __forceinline__ float node_lb(cdx::F3 p, const Node& n) {
  float d2;
  const float l2 = cyl_lb2(p, n.a, n.b, n.m.x, &d2);
  return fmaxf(bsqrt(l2), bsqrt(d2) - n.a.w);
}

__device__ __forceinline__ Node load_node(const Node* __restrict__ p, int i) {
  const float4* q = reinterpret_cast<const float4*>(p + i);
  Node n;
  n.a = q[0]; n.b = q[1]; n.m = q[2];
  return n;
}
__device__ __forceinline__ Slab load_slab(const Slab* __restrict__ p, int64_t i) {
  const float4* q = reinterpret_cast<const float4*>(p + i);
  Slab s;
  s.a = q[0]; s.b = q[1];
  return s;
}

constexpr int REC_WORDS = sizeof(cdx::FaceRec) / 4;  // 40
static_assert(REC_WORDS * CHUNK % (64 * 4) == 0, "a chunk's records load as whole dwordx4 per lane");
constexpr int REC_V4 = REC_WORDS * CHUNK / (64 * 4);   // dwordx4 loads per lane per chunk (5)
static_assert(sizeof(Slab) * CHUNK == 64 * 16, "a chunk's slabs load as one dwordx4 per lane");
#if defined(CDX_SDF_CHUNKS_LDS)
constexpr int NODES_LDS = 512;  // chunk nodes staged in LDS (F ≤ 16 384 faces): 2 waves per SIMD, slower (r05f)
#else
constexpr int NODES_LDS = 0;    // chunk nodes loaded per visited top node (the wave's share, one vector load)
#endif
constexpr int TOPS_LDS = 64;    // top nodes staged in LDS

// (distance, face) as one unsigned 64-bit word whose order is the winner rule's: a non-negative float's
// bits order as unsigned integers, ties then go to the smaller index.
__device__ inline unsigned long long pack_best(float d, int idx) {
  return ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)idx;
}

// One workgroup per 64 Morton-sorted points: its NW waves hold the same 64 points (lane = point) and split
// the work — the greedy seed's tops / chunks / faces NW ways, then the chunks of every top node some lane
// cannot rule out (wave w takes chunks w, w + NW, … of the top) — and share each point's packed best in LDS,
// so a face one wave evaluates tightens the bounds the others test.  Grid: ⌈P/64⌉ workgroups of NW waves.
#ifndef CDX_SDF_NW
#define CDX_SDF_NW 4
#endif
constexpr int NW = CDX_SDF_NW;     // waves per point group
#ifndef CDX_SDF_MINW
#define CDX_SDF_MINW 5  // waves per SIMD the tree kernel is compiled for: 96 VGPRs, 30.7 KB LDS per group → 5 (1: 101 VGPRs, 4)
#endif
constexpr int CPW = TOPB / NW;     // chunks of a top node per wave
static_assert(TOPB % NW == 0 && CHUNK % NW == 0, "waves split a top's chunks and a chunk's faces evenly");
#if defined(CDX_SDF_DIAG)
// timing-only diagnostic: per workgroup [start, end] (s_memrealtime, 100 MHz) of the last tree launch
__device__ unsigned long long g_sdf_wgtime[65536][4];  // start, end, chunk visits, pairs (summed over waves)
#endif
__device__ __forceinline__ void sel_min(float& lb, int& sel, float l, int i) {
  if (l < lb || (l == lb && i < sel)) { lb = l; sel = i; }
}

__device__ __forceinline__ void sdf_tree_body(
    const float* __restrict__ points, int64_t P, const int* __restrict__ porder, const float* __restrict__ faces,
    int64_t F, const cdx::FaceRec* __restrict__ rec, const Slab* __restrict__ slab, const Node* __restrict__ chunk,
    const Node* __restrict__ top, const Node* __restrict__ run, int C, int T, const unsigned* __restrict__ ws,
    float* __restrict__ out_dist,
    int32_t* __restrict__ out_sign, float* __restrict__ out_nrm, float* __restrict__ out_clst,
    int32_t* __restrict__ out_face, int count, int64_t grp) {
  if (ws[6]) return;  // mesh has a NaN-capable face: sdf_exact_kernel does this call
#if defined(CDX_SDF_DIAG)
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
  __shared__ float4 s_rec[NW][REC_WORDS * CHUNK / 4];  // per wave: the visited chunk's face records
  __shared__ float4 s_slab[NW][2 * CHUNK];             // … and its face slabs
  __shared__ float4 s_run[NW][3 * RPC];               // … and its runs' nodes
  __shared__ unsigned long long s_tmask;              // top nodes some lane cannot rule out (T ≤ 64)
  __shared__ float4 s_node[3 * (NODES_LDS + TOPS_LDS)];  // chunk nodes, then top nodes (when they fit)
  __shared__ float4 s_cn[NW][3 * CPW];                // per wave: its CPW chunk nodes of the current top node
  __shared__ unsigned long long s_best[64];           // the group's packed (distance, face) best per point
  __shared__ unsigned short s_pair[NW][128];           // per wave: pending (lane << 5 | face) pairs
  // greedy seed: per wave candidate bound and index — in the record buffers, which the seed phase does not use
  static_assert(sizeof(s_rec) >= NW * 64 * (sizeof(float) + sizeof(int)), "seed scratch fits the record buffers");
  float (*s_lb)[64] = reinterpret_cast<float (*)[64]>(&s_rec[0][0]);
  int (*s_sel)[64] = reinterpret_cast<int (*)[64]>(reinterpret_cast<float*>(&s_rec[0][0]) + NW * 64);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the upper levels of the hierarchy in LDS: one coalesced copy per workgroup instead of a dependent load per
  // node test (the tests then read LDS; a mesh with more nodes reads the rest from global memory)
  const bool chunks_lds = C <= NODES_LDS, tops_lds = T <= TOPS_LDS;
  {
    const float4* cs = reinterpret_cast<const float4*>(chunk);
    const float4* ts = reinterpret_cast<const float4*>(top);
    if (chunks_lds)
      for (int i = threadIdx.x; i < 3 * C; i += 64 * NW) s_node[i] = cs[i];
    if (tops_lds)
      for (int i = threadIdx.x; i < 3 * T; i += 64 * NW) s_node[3 * NODES_LDS + i] = ts[i];
    __syncthreads();
  }
  // the wave's chunks of top node t are t·16 + w + NW·i, i < CPW: staged per wave (one vector load) unless all
  // chunk nodes are in LDS; wave_chunk(t, i) then reads LDS either way
  auto stage_chunks = [&](int t) {
    if (chunks_lds) return;
    if (lane < 3 * CPW) {
      const int c = t * TOPB + w + NW * (lane / 3);
      s_cn[w][lane] = c < C ? reinterpret_cast<const float4*>(chunk)[3 * c + lane % 3] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __builtin_amdgcn_wave_barrier();
  };
  auto wave_chunk = [&](int t, int i) {
    if (chunks_lds) {
      const int c = t * TOPB + w + NW * i;
      return Node{s_node[3 * c], s_node[3 * c + 1], s_node[3 * c + 2]};
    }
    return Node{s_cn[w][3 * i], s_cn[w][3 * i + 1], s_cn[w][3 * i + 2]};
  };
  auto top_node = [&](int t) {
    if (tops_lds) return Node{s_node[3 * (NODES_LDS + t)], s_node[3 * (NODES_LDS + t) + 1], s_node[3 * (NODES_LDS + t) + 2]};
    return load_node(top, t);
  };
  const int64_t j = grp * 64 + lane;
  const bool live0 = j < P;
  const int64_t pi = porder[live0 ? j : P - 1];  // dead lanes shadow a live point
  const cdx::F3 p0 = cdx::f3(points[3 * pi], points[3 * pi + 1], points[3 * pi + 2]);
  const bool ok = fabsf(p0.x) <= PT_LIM && fabsf(p0.y) <= PT_LIM && fabsf(p0.z) <= PT_LIM;
  const unsigned long long badm = __ballot(!ok);  // same points in every wave: uniform over the workgroup
  if (badm) {
#if defined(CDX_SDF_EXACT_GROUP)  // (A/B: the whole group by the tile rule, one point per lane of wave 0)
    if (w == 0) {
      exact_point(p0, faces, F, pi, out_dist, out_sign, out_nrm, out_clst, out_face, live0);
      if (count && lane == 0)
        atomicAdd(&g_sdf_stats[1], (unsigned long long)F * (unsigned long long)__popcll(__ballot(live0)));
    }
    return;
#else
    // a non-finite or out-of-range point (an optimiser's diverged candidate) takes the reference's tile rule, its
    // faces split over the lanes of one wave (the waves take such points in turn); the group's other points walk
    // the tree as usual
    // A point with a NaN coordinate has a NaN distance to every face (p − c carries the NaN), so the rule keeps the
    // first face of the first tile: face 0's point_face, no scan (diverged candidates are mostly NaN, and the sort
    // gathers them into the same groups)
    const bool nanp = p0.x != p0.x || p0.y != p0.y || p0.z != p0.z;
    if (w == 0 && live0 && nanp) {
      cdx::F3 c, n;
      int sg;
      const float d = cdx::point_face(p0, cdx::f3(faces[0], faces[1], faces[2]), cdx::f3(faces[3], faces[4], faces[5]),
                                      cdx::f3(faces[6], faces[7], faces[8]), c, n, sg);
      out_dist[pi] = d;
      out_sign[pi] = sg;
      out_nrm[3 * pi] = n.x; out_nrm[3 * pi + 1] = n.y; out_nrm[3 * pi + 2] = n.z;
      out_clst[3 * pi] = c.x; out_clst[3 * pi + 1] = c.y; out_clst[3 * pi + 2] = c.z;
      if (out_face) out_face[pi] = 0;
    }
    // the others (an infinite or out-of-range coordinate) scan every face (dead lanes shadowing a bad point: nothing
    // to write)
    const unsigned long long todo = badm & __ballot(live0) & ~__ballot(nanp);
    int k = 0;
    for (unsigned long long m = todo; m; m &= m - 1, ++k)
      if (k % NW == w) exact_point_wave(__builtin_ctzll(m), p0, pi, live0, faces, F, out_dist, out_sign, out_nrm,
                                        out_clst, out_face);
    if (count && threadIdx.x == 0)  // (the brute-force pairs the tile rule stands for, NaN points included)
      atomicAdd(&g_sdf_stats[1], (unsigned long long)F * (unsigned long long)__popcll(badm & __ballot(live0)));
    if (!~badm) return;
#endif
  }
  // the walk: a bad lane shadows the first good lane's point and writes nothing
  const int sh = __builtin_ctzll(~badm);
  const cdx::F3 p = ok ? p0 : cdx::f3(__shfl(p0.x, sh), __shfl(p0.y, sh), __shfl(p0.z, sh));
  const bool live = live0 && ok;
  const float pnorm = bsqrt(p.x * p.x + p.y * p.y + p.z * p.z);
  // merge the four waves' (bound, index) candidates: the smallest bound, then the smallest index
  auto merge = [&](float lb, int sel) {
    s_lb[w][lane] = lb;
    s_sel[w][lane] = sel;
    __syncthreads();
    float m = s_lb[0][lane];
    int si = s_sel[0][lane];
#pragma unroll
    for (int v = 1; v < NW; ++v) sel_min(m, si, s_lb[v][lane], s_sel[v][lane]);
    __syncthreads();
    return si;
  };

  // greedy seed: nearest top node, nearest chunk in it, the face of smallest slab bound in that chunk —
  // evaluated exactly, so every point starts with a real (distance, face) near its answer
  int tsel;
  {
    float tl = INFINITY;
    int ts = 0x7fffffff;
    for (int t = w; t < T; t += NW) sel_min(tl, ts, node_lb(p, top_node(t)), t);
    tsel = merge(tl, ts);
    if (tsel >= T) tsel = 0;
  }
  int csel;
  {
    float cl = INFINITY;
    int cs = 0x7fffffff;
    if (!chunks_lds) {  // (a per-lane top: each lane loads its own 4 nodes)
      for (int i = 0; i < CPW; ++i) {
        const int c = tsel * TOPB + w + NW * i;
        if (c < C) sel_min(cl, cs, node_lb(p, load_node(chunk, c)), c);
      }
    } else {
      for (int i = 0; i < CPW; ++i) {
        const int c = tsel * TOPB + w + NW * i;
        if (c < C) sel_min(cl, cs, node_lb(p, Node{s_node[3 * c], s_node[3 * c + 1], s_node[3 * c + 2]}), c);
      }
    }
    csel = merge(cl, cs);
    if (csel >= C) csel = tsel * TOPB;
  }
  {
    float fl = INFINITY;
    int fs = 0x7fffffff;
    for (int i = 0; i < CHUNK / NW; ++i) {
      const int64_t f = (int64_t)csel * CHUNK + w + NW * i;
      if (f < F) {
        const Slab sl = load_slab(slab, f);
        float d2;
        sel_min(fl, fs, cyl_lb2(p, sl.a, sl.b, sl.a.w, &d2), (int)f);
      }
    }
    const int fsel = merge(fl, fs);
    if (w == 0) {
      const cdx::FaceRec r = rec[fsel < F ? fsel : csel * CHUNK];
      s_best[lane] = pack_best(cdx::face_dist2(p, r), r.idx);
    }
    __syncthreads();
  }
  unsigned visits = 0, pairs = 0;
  auto best_now = [&]() { return __uint_as_float((unsigned)(s_best[lane] >> 32)); };

  const float4* rec4 = reinterpret_cast<const float4*>(rec);
  float4* buf = s_rec[w];
  const cdx::FaceRec* rr = reinterpret_cast<const cdx::FaceRec*>(buf);
  // the top nodes some lane cannot rule out against the seeds, tested once per workgroup (waves split them) when
  // they fit one mask word; each is re-tested against the current best before its chunks are walked
#if defined(CDX_SDF_NO_TMASK)
  const bool shared_tops = false;
#else
  const bool shared_tops = tops_lds && T <= 64;
#endif
  if (shared_tops) {
    if (threadIdx.x == 0) s_tmask = 0ull;
    __syncthreads();
    const float sb0 = bsqrt(best_now());
    for (int t = w; t < T; t += NW)
      if (__any(node_needed(p, top_node(t), sb0, pnorm)) && lane == 0) atomicOr(&s_tmask, 1ull << t);
    __syncthreads();
  }
  const unsigned long long tmask = shared_tops ? s_tmask : ~0ull;
  for (int t = 0; t < T; ++t) {
    if (shared_tops && !((tmask >> t) & 1ull)) continue;
    if (!__any(node_needed(p, top_node(t), bsqrt(best_now()), pnorm))) continue;
    stage_chunks(t);
    for (int i = 0; i < CPW; ++i) {
      const int c = t * TOPB + w + NW * i;
      if (c >= C) break;
      const Node cn = wave_chunk(t, i);
      const float sb = bsqrt(best_now());
      if (!__any(node_needed(p, cn, sb, pnorm))) continue;
      // the chunk's face slabs (one dwordx4 per lane) and records (5 per lane) in flight together, into the
      // wave's LDS buffers
      {
        static_assert(REC_V4 == 5, "five record loads per lane");
        const float4* rc = rec4 + (int64_t)c * (REC_WORDS * CHUNK / 4) + lane;
#if defined(CDX_SDF_REG_STAGE)  // (A/B: through registers — 28 VGPRs in flight)
        const float4 v0 = rc[0], v1 = rc[64], v2 = rc[128], v3 = rc[192], v4 = rc[256];
        const float4 sv = reinterpret_cast<const float4*>(slab)[(int64_t)c * 2 * CHUNK + lane];
        const float4 rv = lane < 3 * RPC ? reinterpret_cast<const float4*>(run)[(int64_t)c * 3 * RPC + lane]
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
        __builtin_amdgcn_wave_barrier();
        s_slab[w][lane] = sv;
        if (lane < 3 * RPC) s_run[w][lane] = rv;
        buf[lane] = v0; buf[lane + 64] = v1; buf[lane + 128] = v2; buf[lane + 192] = v3; buf[lane + 256] = v4;
        __builtin_amdgcn_wave_barrier();
#else  // LDS-DMA (global_load_lds_dwordx4: lane l's 16 bytes to base + 16·l, no VGPRs, no ds_write)
        typedef __attribute__((address_space(3))) void* lds_ptr;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the previous chunk's LDS reads are done)
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const float4*>(slab) + (int64_t)c * 2 * CHUNK + lane,
                                         (lds_ptr)&s_slab[w][0], 16, 0, 0);
        if (lane < 3 * RPC)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const float4*>(run) + (int64_t)c * 3 * RPC + lane,
                                           (lds_ptr)&s_run[w][0], 16, 0, 0);
#pragma unroll
        for (int q = 0; q < REC_V4; ++q) __builtin_amdgcn_global_load_lds(rc + 64 * q, (lds_ptr)(buf + 64 * q), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#endif
      }
      // the chunk's faces a lane cannot rule out: the runs first (their own nodes), then the slab bound of each
      // face of a run some lane needs, against the chunk's threshold (its margins)
      const float th = node_th(cn, sb, pnorm);
      const float th2 = th * th;
      const int nf = (int)min((int64_t)CHUNK, F - (int64_t)c * CHUNK);
      unsigned lmask = 0;
#pragma unroll
      for (int rr = 0; rr < RPC; ++rr) {
        if (rr * RUN >= nf) break;
#if !defined(CDX_SDF_NO_RUNS)
        const Node rn = Node{s_run[w][3 * rr], s_run[w][3 * rr + 1], s_run[w][3 * rr + 2]};
        if (!__any(node_needed(p, rn, sb, pnorm))) continue;
#endif
#pragma unroll
        for (int kk = 0; kk < RUN; ++kk) {
          const int k = RUN * rr + kk;
          const float4 sa = s_slab[w][2 * k], sbv = s_slab[w][2 * k + 1];
          float d2;
          const float l2 = cyl_lb2(p, sa, sbv, sa.w, &d2);
          if (!(l2 > th2) && k < nf && live) lmask |= 1u << k;
        }
      }
      unsigned mask = lmask;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mask |= (unsigned)__shfl_xor((int)mask, o);
      mask = __builtin_amdgcn_readfirstlane(mask);
      if (!mask) continue;
      ++visits;
      // the (lane, face) pairs, packed 64 to a round: lane i of a round evaluates pair i (its point read from
      // the owner) and folds it into the owner's packed best with an LDS 64-bit minimum (the winner order)
      auto eval_round = [&](int n) {
        const unsigned e = s_pair[w][lane];
        const int l = lane < n ? (int)(e >> 5) : lane;
        const float qx = __shfl(p.x, l), qy = __shfl(p.y, l), qz = __shfl(p.z, l);
        if (lane < n) {
          const cdx::FaceRec& r = rr[e & 31u];
          atomicMin(&s_best[l], pack_best(cdx::face_dist2(cdx::f3(qx, qy, qz), r), r.idx));
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
          __builtin_amdgcn_wave_barrier();
          eval_round(64);
          cnt -= 64;
          const unsigned short tail = s_pair[w][64 + lane];  // (read before any lane overwrites its slot)
          __builtin_amdgcn_wave_barrier();
          if (lane < cnt) s_pair[w][lane] = tail;
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (cnt > 0) eval_round(cnt);
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (count) {
    const unsigned long long nl = __popcll(__ballot(live));
    if (lane == 0) {
      atomicAdd(&g_sdf_stats[0], (unsigned long long)pairs + (w == 0 ? nl : 0ull));
      if (w == 0) atomicAdd(&g_sdf_stats[2], nl);
      atomicAdd(&g_sdf_stats[3], (unsigned long long)visits);
    }
  }
#if defined(CDX_SDF_DIAG)
  __shared__ unsigned s_diag[2];
  if (threadIdx.x == 0) s_diag[0] = s_diag[1] = 0u;
  __syncthreads();
  if (lane == 0) { atomicAdd(&s_diag[0], visits); atomicAdd(&s_diag[1], pairs); }
#endif
  __syncthreads();
#if defined(CDX_SDF_DIAG)
  if (threadIdx.x == 0 && blockIdx.x < 65536) {
    g_sdf_wgtime[blockIdx.x][0] = t_start;
    g_sdf_wgtime[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
    g_sdf_wgtime[blockIdx.x][2] = s_diag[0];
    g_sdf_wgtime[blockIdx.x][3] = s_diag[1];
  }
#endif
  if (w != 0 || !live) return;
  const int bidx = (int)(unsigned)s_best[lane];
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

__global__ __launch_bounds__(64 * NW, CDX_SDF_MINW) void sdf_tree_kernel(
    const float* __restrict__ points, int64_t P, const int* __restrict__ porder, const float* __restrict__ faces,
    int64_t F, const cdx::FaceRec* __restrict__ rec, const Slab* __restrict__ slab, const Node* __restrict__ chunk,
    const Node* __restrict__ top, const Node* __restrict__ run, int C, int T, const unsigned* __restrict__ ws,
    float* __restrict__ out_dist, int32_t* __restrict__ out_sign, float* __restrict__ out_nrm,
    float* __restrict__ out_clst, int32_t* __restrict__ out_face, int count) {
  sdf_tree_body(points, P, porder, faces, F, rec, slab, chunk, top, run, C, T, ws, out_dist, out_sign, out_nrm, out_clst,
                out_face, count, blockIdx.x);
}

// Several queries (ordered, culled meshes) in one launch: workgroup b runs point group b − first[q] of query q.  The
// queries' tails (the few groups far from each mesh) overlap in one grid, with no stream or event between them.
constexpr int SDF_BATCH_MAX = 4;
struct SdfBatchQ {
  const float* points;
  int64_t P;
  const int* porder;
  const float* faces;
  int64_t F;
  const cdx::FaceRec* rec;
  const Slab* slab;
  const Node *chunk, *top, *run;
  int C, T;
  const unsigned* ws;
  float* out_dist;
  int32_t* out_sign;
  float *out_nrm, *out_clst;
  int32_t* out_face;
};
struct SdfBatch {
  SdfBatchQ q[SDF_BATCH_MAX];
  unsigned first[SDF_BATCH_MAX];
  int n, count;
  unsigned* sched;  // nullable: the launch schedule (below)
  unsigned cap;     // groups the schedule holds
};
// Launch schedule of a batch (cdx_sdf_query_batch's `schedule`, uint32 words): [0] the group count the order below
// is for (0: none yet), [1..3] reserved, cost[cap] (each group's duration in the last launch, 100 MHz ticks),
// order[cap] (a permutation of the groups: heaviest first).  A group's walk time spreads 2-3× (the groups far from a
// mesh test many more nodes); dispatched in point order, the heavy groups that start last set the launch's end.
// Workgroup b runs group order[b], so the heaviest groups of the previous launch — the same points, or points a sort
// later, an optimiser step away — start first and the light ones fill the tail.  Any permutation gives the same
// outputs: every group writes only its own points.
constexpr int SDF_SCHED_HDR = 4;
__global__ __launch_bounds__(64 * NW, CDX_SDF_MINW) void sdf_tree_batch_kernel(SdfBatch b) {
  // the descriptors read in place from the kernel-argument segment (indexed per workgroup, a by-value copy would go
  // to scratch)
  const SdfBatch& kb = *(const SdfBatch*)(__builtin_amdgcn_kernarg_segment_ptr());
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned grp = blockIdx.x;
  if (kb.sched && kb.sched[0] == gridDim.x) {
    const unsigned v = kb.sched[SDF_SCHED_HDR + kb.cap + blockIdx.x];
    grp = v < gridDim.x ? v : grp;
  }
  grp = __builtin_amdgcn_readfirstlane(grp);
  int qi = 0;
#pragma unroll
  for (int i = 1; i < SDF_BATCH_MAX; ++i)
    if (i < kb.n && grp >= kb.first[i]) qi = i;
  qi = __builtin_amdgcn_readfirstlane(qi);
  const SdfBatchQ& q = kb.q[qi];
  sdf_tree_body(q.points, q.P, q.porder, q.faces, q.F, q.rec, q.slab, q.chunk, q.top, q.run, q.C, q.T, q.ws,
                q.out_dist, q.out_sign, q.out_nrm, q.out_clst, q.out_face, kb.count, (int64_t)grp - kb.first[qi]);
  if (kb.sched && threadIdx.x == 0)  // (after the body's last barrier: every wave's walk is done)
    kb.sched[SDF_SCHED_HDR + grp] = (unsigned)(__builtin_amdgcn_s_memrealtime() - t0);
}

// The next launch's order from this launch's group durations: a counting sort on SCHED_BINS duration bins, heaviest
// bin first (one workgroup; the order inside a bin is whatever the LDS atomics give — any order is correct).
constexpr int SCHED_BINS = 64, SCHED_THREADS = 1024;
__global__ __launch_bounds__(SCHED_THREADS) void sdf_batch_sched_kernel(unsigned* __restrict__ sch, unsigned G,
                                                                        unsigned cap) {
  __shared__ unsigned s_hist[SCHED_BINS], s_max;
  const unsigned* cost = sch + SDF_SCHED_HDR;
  unsigned* order = sch + SDF_SCHED_HDR + cap;
  const unsigned t = threadIdx.x;
  if (t < SCHED_BINS) s_hist[t] = 0u;
  if (t == 0) s_max = 0u;
  __syncthreads();
  unsigned m = 0u;
  for (unsigned g = t; g < G; g += SCHED_THREADS) m = max(m, cost[g]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  if ((t & 63) == 0) atomicMax(&s_max, m);
  __syncthreads();
  const unsigned long long span = (unsigned long long)s_max + 1ull;
  auto bin = [&](unsigned c) { return (unsigned)(SCHED_BINS - 1) - (unsigned)((unsigned long long)c * SCHED_BINS / span); };
  for (unsigned g = t; g < G; g += SCHED_THREADS) atomicAdd(&s_hist[bin(cost[g])], 1u);
  __syncthreads();
  if (t == 0) {  // exclusive prefix: each bin's first position
    unsigned acc = 0u;
    for (int i = 0; i < SCHED_BINS; ++i) {
      const unsigned c = s_hist[i];
      s_hist[i] = acc;
      acc += c;
    }
  }
  __syncthreads();
  for (unsigned g = t; g < G; g += SCHED_THREADS) order[atomicAdd(&s_hist[bin(cost[g])], 1u)] = g;
  if (t == 0) sch[0] = G;
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

bool sched_on() {  // CDX_SDF_SCHED=0: a batch ignores its schedule (point order, the A/B base)
  static const bool on = [] {
    const char* e = cdx::ab_env("CDX_SDF_SCHED");
    return !(e && e[0] == '0');
  }();
  return on;
}

int sdf_mode() {  // CDX_SDF_MODE=exact forces the brute-force kernel (benchmarks, A/B tests)
  static const int m = [] {
    const char* e = cdx::ab_env("CDX_SDF_MODE");
    return (e && e[0] == 'e') ? 1 : 0;
  }();
  return m;
}


// Mesh: [header words: frame keys ×6, may-NaN flag, 0][face records: C·CHUNK FaceRec][slabs: C·CHUNK Slab]
// [chunk nodes: C Node][top nodes: T Node], C = ⌈F/32⌉, T = ⌈C/16⌉, faces in the build's order.
int64_t n_chunks(int64_t F) { return (F + CHUNK - 1) / CHUNK; }
// (runs: RUN-face groups of a chunk, RPC per chunk, each with its own node — tested before the run's faces)
int64_t n_tops(int64_t F) { return (n_chunks(F) + TOPB - 1) / TOPB; }
size_t mesh_rec_off() { return align256(8 * sizeof(unsigned)); }
size_t mesh_slab_off(int64_t C) { return mesh_rec_off() + align256((size_t)C * CHUNK * sizeof(cdx::FaceRec)); }
size_t mesh_chunk_off(int64_t C) { return mesh_slab_off(C) + align256((size_t)C * CHUNK * sizeof(Slab)); }
size_t mesh_top_off(int64_t C) { return mesh_chunk_off(C) + align256((size_t)C * sizeof(Node)); }
size_t mesh_run_off(int64_t C) { return mesh_top_off(C) + align256((size_t)((C + TOPB - 1) / TOPB) * sizeof(Node)); }
size_t mesh_bytes(int64_t F) {
  const int64_t C = n_chunks(F);
  return mesh_run_off(C) + align256((size_t)C * RPC * sizeof(Node));
}

// Records, slabs and nodes of the faces in `order` (device int[F]).
void mesh_fill(const float* faces, int64_t F, const int* order, char* mesh, hipStream_t s) {
  const int64_t C = n_chunks(F), T = n_tops(F);
  unsigned* ws = reinterpret_cast<unsigned*>(mesh);
  auto* rec = reinterpret_cast<cdx::FaceRec*>(mesh + mesh_rec_off());
  hipLaunchKernelGGL(sdf_face_kernel, dim3((unsigned)((C * CHUNK + 255) / 256)), dim3(256), 0, s, faces, F,
                     (int64_t)(C * CHUNK), order, rec, reinterpret_cast<Slab*>(mesh + mesh_slab_off(C)), ws);
  hipLaunchKernelGGL(sdf_node_kernel, dim3((unsigned)C), dim3(64), 0, s, (const cdx::FaceRec*)rec, F, CHUNK,
                     reinterpret_cast<Node*>(mesh + mesh_chunk_off(C)));
  hipLaunchKernelGGL(sdf_node_kernel, dim3((unsigned)T), dim3(64), 0, s, (const cdx::FaceRec*)rec, F, CHUNK * TOPB,
                     reinterpret_cast<Node*>(mesh + mesh_top_off(C)));
  hipLaunchKernelGGL(sdf_node_kernel, dim3((unsigned)(C * RPC)), dim3(64), 0, s, (const cdx::FaceRec*)rec, F, RUN,
                     reinterpret_cast<Node*>(mesh + mesh_run_off(C)));
}

// One-shot build on the device: face centroids in Morton order (10 bits per axis) of the faces' cubic frame.
int mesh_build_morton(const float* faces, int64_t F, char* mesh, hipStream_t s) {
  const int n = (int)F;
  size_t tf = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tf, (unsigned*)nullptr, (unsigned*)nullptr, (int*)nullptr,
                                         (int*)nullptr, n, 0, 30, s) != hipSuccess)
    return CDX_ELAUNCH;
  size_t off = 0;
  const size_t o_part = off; off = align256(off + 6 * BBOX_BLOCKS * sizeof(unsigned));
  const size_t o_fk = off; off = align256(off + 2 * (size_t)n * sizeof(unsigned));
  const size_t o_fv = off; off = align256(off + 2 * (size_t)n * sizeof(int));
  const size_t o_tmp = off; off = align256(off + tf);
  char* base = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&base), off, s) != hipSuccess) return CDX_ELAUNCH;
  unsigned* ws = reinterpret_cast<unsigned*>(mesh);
  unsigned* part = reinterpret_cast<unsigned*>(base + o_part);
  unsigned* fk = reinterpret_cast<unsigned*>(base + o_fk);
  int* fv = reinterpret_cast<int*>(base + o_fv);
  const int nb = (int)std::min<int64_t>((3 * F + 255) / 256, BBOX_BLOCKS);
  hipLaunchKernelGGL(sdf_bbox_kernel, dim3(nb), dim3(256), 0, s, faces, 3 * F, part, ws + 6);
  hipLaunchKernelGGL(sdf_keys_kernel, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, s, faces, F, 1,
                     (const unsigned*)part, nb, 10, fk, fv);
  size_t t1 = tf;
  bool ok = hipcub::DeviceRadixSort::SortPairs(base + o_tmp, t1, fk, fk + n, fv, fv + n, n, 0, 30, s) == hipSuccess;
  mesh_fill(faces, F, fv + n, mesh, s);
  ok = ok && hipGetLastError() == hipSuccess;
  ok = (hipFreeAsync(base, s) == hipSuccess) && ok;
  return ok ? CDX_OK : CDX_ELAUNCH;
}

// Face order of a median-split k-d tree on the centroids: split the longest extent of the node's centroids at
// a left size that is a multiple of a top node (512 faces) while the node is larger than one, else of a chunk
// (32), else of a run (8), so every run, chunk and top node is one subtree (a compact cluster).
void kd_order(const std::vector<float>& cen, std::vector<int>& idx) {
  struct Range { int lo, hi; };
  std::vector<Range> stack{{0, (int)idx.size()}};
  while (!stack.empty()) {
    const Range r = stack.back();
    stack.pop_back();
    const int n = r.hi - r.lo;
    if (n <= RUN) continue;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = r.lo; i < r.hi; ++i)
      for (int c = 0; c < 3; ++c) {
        const float v = cen[3 * (size_t)idx[i] + c];
        if (v < lo[c]) lo[c] = v;
        if (v > hi[c]) hi[c] = v;
      }
    int ax = 0;
    for (int c = 1; c < 3; ++c)
      if (hi[c] - lo[c] > hi[ax] - lo[ax]) ax = c;
    const int unit = n > CHUNK * TOPB ? CHUNK * TOPB : (n > CHUNK ? CHUNK : RUN);
    const int half = std::min(((n + 1) / 2 + unit - 1) / unit * unit, n - 1);
    std::nth_element(idx.begin() + r.lo, idx.begin() + r.lo + half, idx.begin() + r.hi, [&](int a, int b) {
      const float ka = cen[3 * (size_t)a + ax], kb = cen[3 * (size_t)b + ax];
      return ka < kb || (ka == kb && a < b);  // (NaN centroids: any consistent side is fine for the order)
    });
    stack.push_back({r.lo, r.lo + half});
    stack.push_back({r.lo + half, r.hi});
  }
}

// Prepared build: the k-d order on the host (one device→host copy of the faces and a wait on the stream),
// then the records and nodes on the device.
int mesh_build_kd(const float* faces, int64_t F, char* mesh, hipStream_t s) {
  std::vector<float> fh((size_t)F * 9);
  if (hipMemcpyAsync(fh.data(), faces, fh.size() * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CDX_ELAUNCH;
  std::vector<float> cen((size_t)F * 3);
  for (int64_t f = 0; f < F; ++f)
    for (int c = 0; c < 3; ++c) {
      const float* v = &fh[9 * (size_t)f];
      cen[3 * (size_t)f + c] = (v[c] + v[3 + c] + v[6 + c]) / 3.f;
    }
  std::vector<int> idx((size_t)F);
  for (int64_t f = 0; f < F; ++f) idx[(size_t)f] = (int)f;
  kd_order(cen, idx);
  int* order = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&order), (size_t)F * sizeof(int), s) != hipSuccess) return CDX_ELAUNCH;
  bool ok = hipMemcpyAsync(order, idx.data(), (size_t)F * sizeof(int), hipMemcpyHostToDevice, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess;  // (idx is freed on return)
  hipLaunchKernelGGL(sdf_init_kernel, dim3(1), dim3(64), 0, s, reinterpret_cast<unsigned*>(mesh));  // (may-NaN flag)
  mesh_fill(faces, F, order, mesh, s);
  ok = ok && hipGetLastError() == hipSuccess;
  ok = (hipFreeAsync(order, s) == hipSuccess) && ok;
  return ok ? CDX_OK : CDX_ELAUNCH;
}

// Query workspace: [bbox partials 6·BBOX_BLOCKS words][keys 2P][values 2P][radix-sort scratch]; the points' order
// stays at values + P for a later query of the same points (CDX_SDF_REUSE_ORDER).
constexpr int POINT_MB = 6;  // Morton bits per axis of the point order (64³ cells over the points' box; finer
                             // levels only reorder points within a wave's neighbourhood)
struct QueryWs { size_t o_pk, o_pv, o_tmp, bytes, tp; };
bool query_ws(int64_t P, hipStream_t s, QueryWs& q) {
  const int m = (int)P;
  q.tp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, q.tp, (unsigned*)nullptr, (unsigned*)nullptr, (int*)nullptr,
                                         (int*)nullptr, m, 0, 3 * POINT_MB, s) != hipSuccess)
    return false;
  size_t off = align256(6 * BBOX_BLOCKS * sizeof(unsigned));
  q.o_pk = off; off = align256(off + 2 * (size_t)m * sizeof(unsigned));
  q.o_pv = off; off = align256(off + 2 * (size_t)m * sizeof(int));
  q.o_tmp = off; off = align256(off + q.tp);
  q.bytes = off;
  return true;
}

// Points in Morton order of their own cubic frame (a workgroup then holds nearby points; skipped with
// CDX_SDF_REUSE_ORDER), the tree kernel (skipped with CDX_SDF_MESH_EXACT), and the brute-force tile rule when the
// mesh may produce NaN distances (decided on the device; skipped with CDX_SDF_MESH_CULLED).
// The points' Morton order into workspace `base` (bbox partials, keys, an 18-bit radix sort): the order stays at
// values + P for the tree kernel of this and later CDX_SDF_REUSE_ORDER queries.
bool mesh_order(const float* points, int64_t P, char* base, const QueryWs& q, hipStream_t s) {
  const int m = (int)P;
  unsigned* part = reinterpret_cast<unsigned*>(base);
  unsigned* pk = reinterpret_cast<unsigned*>(base + q.o_pk);
  int* pv = reinterpret_cast<int*>(base + q.o_pv);
  const int nb = (int)std::min<int64_t>((P + 255) / 256, BBOX_BLOCKS);
  hipLaunchKernelGGL(sdf_bbox_kernel, dim3(nb), dim3(256), 0, s, points, P, part, (unsigned*)nullptr);
  hipLaunchKernelGGL(sdf_keys_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, points, P, 0,
                     (const unsigned*)part, nb, POINT_MB, pk, pv);
  size_t t2 = q.tp;
  return hipcub::DeviceRadixSort::SortPairs(base + q.o_tmp, t2, pk, pk + m, pv, pv + m, m, 0, 3 * POINT_MB, s) ==
             hipSuccess &&
         hipGetLastError() == hipSuccess;
}

int mesh_query(const char* mesh, const float* faces, int64_t F, const float* points, int64_t P, float* sqdist,
               int32_t* sign, float* normals, float* clst, int32_t* face_idx, char* base, const QueryWs& q, int flags,
               hipStream_t s) {
  const int m = (int)P;
  const int64_t C = n_chunks(F), T = n_tops(F);
  const unsigned* mws = reinterpret_cast<const unsigned*>(mesh);
  int* pv = reinterpret_cast<int*>(base + q.o_pv);
  bool ok = true;
  if (!(flags & CDX_SDF_REUSE_ORDER) && !(flags & CDX_SDF_MESH_EXACT)) ok = mesh_order(points, P, base, q, s);
  if (!(flags & CDX_SDF_MESH_EXACT))
    hipLaunchKernelGGL(sdf_tree_kernel, dim3((unsigned)((P + 63) / 64)), dim3(64 * NW), 0, s, points, P,
                       (const int*)(pv + m), faces, F, reinterpret_cast<const cdx::FaceRec*>(mesh + mesh_rec_off()),
                       reinterpret_cast<const Slab*>(mesh + mesh_slab_off(C)),
                       reinterpret_cast<const Node*>(mesh + mesh_chunk_off(C)),
                       reinterpret_cast<const Node*>(mesh + mesh_top_off(C)),
                       reinterpret_cast<const Node*>(mesh + mesh_run_off(C)), (int)C, (int)T, mws, sqdist, sign,
                       normals, clst, face_idx, (int)g_sdf_count);
  if (!(flags & CDX_SDF_MESH_CULLED))
    hipLaunchKernelGGL(sdf_exact_kernel, dim3((unsigned)((P + SDF_BLOCK - 1) / SDF_BLOCK)), dim3(SDF_BLOCK), 0, s,
                       points, P, faces, F, mws, sqdist, sign, normals, clst, face_idx, (int)g_sdf_count);
  ok = ok && hipGetLastError() == hipSuccess;
  return ok ? CDX_OK : CDX_ELAUNCH;
}

// mesh_query with workspace `ws` (ws_bytes ≥ cdx_sdf_query_workspace(P)), or stream-ordered scratch when ws is
// NULL (then the order cannot be reused).
int mesh_query_ws(const char* mesh, const float* faces, int64_t F, const float* points, int64_t P, float* sqdist,
                  int32_t* sign, float* normals, float* clst, int32_t* face_idx, void* ws, size_t ws_bytes, int flags,
                  hipStream_t s) {
  QueryWs q;
  if (!query_ws(P, s, q)) return CDX_ELAUNCH;
  if (ws) {
    if (ws_bytes < q.bytes) return CDX_EINVAL;
    return mesh_query(mesh, faces, F, points, P, sqdist, sign, normals, clst, face_idx, static_cast<char*>(ws), q,
                      flags, s);
  }
  if (flags & CDX_SDF_REUSE_ORDER) return CDX_EINVAL;
  char* base = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&base), q.bytes, s) != hipSuccess) return CDX_ELAUNCH;
  int rc = mesh_query(mesh, faces, F, points, P, sqdist, sign, normals, clst, face_idx, base, q, flags, s);
  if (hipFreeAsync(base, s) != hipSuccess && !rc) rc = CDX_ELAUNCH;
  return rc;
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
  int rc = mesh_build_morton(faces, F, mesh, s);
  if (!rc) rc = mesh_query_ws(mesh, faces, F, points, P, sqdist, sign, normals, clst, face_idx, nullptr, 0, 0, s);
  if (hipFreeAsync(mesh, s) != hipSuccess && !rc) rc = CDX_ELAUNCH;
  return rc;
}

size_t cdx_sdf_mesh_bytes(int64_t F) { return F > 0 && F <= INT32_MAX / 9 ? mesh_bytes(F) : 0; }

int cdx_sdf_mesh_prepare(const float* faces, int64_t F, void* mesh, cdx_stream_t stream) {
  if (F <= 0 || F > INT32_MAX / 9 || !faces || !mesh) return CDX_EINVAL;
  return mesh_build_kd(faces, F, static_cast<char*>(mesh), reinterpret_cast<hipStream_t>(stream));
}

size_t cdx_sdf_query_workspace(int64_t P) {
  if (P <= 0 || P > INT32_MAX) return 0;
  QueryWs q;
  return query_ws(P, nullptr, q) ? q.bytes : 0;
}

int cdx_sdf_mesh_flags(const void* mesh, int32_t* flags, cdx_stream_t stream) {
  if (!mesh || !flags) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  unsigned w = 0;
  if (hipMemcpyAsync(&w, static_cast<const unsigned*>(mesh) + 6, sizeof(unsigned), hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CDX_ELAUNCH;
  *flags = w ? CDX_SDF_MESH_EXACT : CDX_SDF_MESH_CULLED;
  return CDX_OK;
}

int cdx_sdf_query(const void* mesh, const float* faces, int64_t F, const float* points, int64_t P, float* sqdist,
                  int32_t* sign, float* normals, float* clst, int32_t* face_idx, void* workspace,
                  size_t workspace_bytes, int32_t flags, cdx_stream_t stream) {
  if (P < 0 || F < 0 || !mesh || (flags & ~7) || (flags & 6) == 6) return CDX_EINVAL;
  if (P == 0) return CDX_OK;
  if (!sdf_args_ok(P, points, faces, F, sqdist, sign, normals, clst)) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (sdf_mode() == 1) return cdx_sdf_forward(points, P, faces, F, sqdist, sign, normals, clst, face_idx, stream);
  return mesh_query_ws(static_cast<const char*>(mesh), faces, F, points, P, sqdist, sign, normals, clst, face_idx,
                       workspace, workspace_bytes, flags, s);
}

#if defined(CDX_SDF_DIAG)
int cdx_sdf_diag_wgtime(uint64_t* out, int64_t n, cdx_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (n > 65536 || hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(g_sdf_wgtime), (size_t)n * 32, 0, hipMemcpyDeviceToHost, s) !=
                       hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return CDX_ELAUNCH;
  return CDX_OK;
}
#endif

size_t cdx_sdf_batch_schedule_bytes(int32_t n, const int64_t* P) {
  if (n < 0 || n > SDF_BATCH_MAX || (n > 0 && !P)) return 0;
  uint64_t groups = 0;
  for (int i = 0; i < n; ++i) {
    if (P[i] < 0 || P[i] > INT32_MAX) return 0;
    groups += (uint64_t)((P[i] + 63) / 64);
  }
  return (size_t)(SDF_SCHED_HDR + 2 * groups) * sizeof(unsigned);
}

int cdx_sdf_query_batch(int32_t n, const cdx_sdf_batch_query* qs, void* schedule, size_t schedule_bytes,
                        cdx_stream_t stream) {
  if (n < 0 || n > SDF_BATCH_MAX || (n > 0 && !qs)) return CDX_EINVAL;
  SdfBatch b{};
  unsigned groups = 0;
  int m = 0;
  for (int i = 0; i < n; ++i) {
    const cdx_sdf_batch_query& d = qs[i];
    const int32_t fl = i == 0 ? (d.flags & ~CDX_SDF_SCHED_KEEP) : d.flags;
    if (d.P < 0 || d.F < 0 || !d.mesh || fl != (CDX_SDF_REUSE_ORDER | CDX_SDF_MESH_CULLED)) return CDX_EINVAL;
    if (d.P == 0) continue;
    if (!sdf_args_ok(d.P, d.points, d.faces, d.F, d.sqdist, d.sign, d.normals, d.clst) || !d.workspace) return CDX_EINVAL;
    QueryWs q;
    if (!query_ws(d.P, reinterpret_cast<hipStream_t>(stream), q)) return CDX_ELAUNCH;
    if (d.workspace_bytes < q.bytes) return CDX_EINVAL;
    const char* mesh = static_cast<const char*>(d.mesh);
    const int64_t C = n_chunks(d.F), T = n_tops(d.F);
    SdfBatchQ& o = b.q[m];
    o.points = d.points;
    o.P = d.P;
    o.porder = reinterpret_cast<const int*>(static_cast<const char*>(d.workspace) + q.o_pv) + d.P;
    o.faces = d.faces;
    o.F = d.F;
    o.rec = reinterpret_cast<const cdx::FaceRec*>(mesh + mesh_rec_off());
    o.slab = reinterpret_cast<const Slab*>(mesh + mesh_slab_off(C));
    o.chunk = reinterpret_cast<const Node*>(mesh + mesh_chunk_off(C));
    o.top = reinterpret_cast<const Node*>(mesh + mesh_top_off(C));
    o.run = reinterpret_cast<const Node*>(mesh + mesh_run_off(C));
    o.C = (int)C;
    o.T = (int)T;
    o.ws = reinterpret_cast<const unsigned*>(mesh);
    o.out_dist = d.sqdist;
    o.out_sign = d.sign;
    o.out_nrm = d.normals;
    o.out_clst = d.clst;
    o.out_face = d.face_idx;
    b.first[m] = groups;
    groups += (unsigned)((d.P + 63) / 64);
    ++m;
  }
  if (m == 0) return CDX_OK;
  b.n = m;
  b.count = (int)g_sdf_count;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (sdf_mode() == 1) {  // (the exact-path debug mode: one call per query)
    for (int i = 0; i < n; ++i) {
      const cdx_sdf_batch_query& d = qs[i];
      const int rc = cdx_sdf_forward(d.points, d.P, d.faces, d.F, d.sqdist, d.sign, d.normals, d.clst, d.face_idx, stream);
      if (rc) return rc;
    }
    return CDX_OK;
  }
  if (schedule && sched_on()) {
    if (schedule_bytes < (size_t)(SDF_SCHED_HDR + 2 * (size_t)groups) * sizeof(unsigned)) return CDX_EINVAL;
    b.sched = static_cast<unsigned*>(schedule);
    b.cap = groups;
  }
  hipLaunchKernelGGL(sdf_tree_batch_kernel, dim3(groups), dim3(64 * NW), 0, s, b);
  if (b.sched && !(qs[0].flags & CDX_SDF_SCHED_KEEP))
    hipLaunchKernelGGL(sdf_batch_sched_kernel, dim3(1), dim3(SCHED_THREADS), 0, s, b.sched, groups, b.cap);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}

int cdx_sdf_query_order(const float* points, int64_t P, void* workspace, size_t workspace_bytes, cdx_stream_t stream) {
  if (P < 0 || P > INT32_MAX) return CDX_EINVAL;
  if (P == 0) return CDX_OK;
  if (!points || !workspace) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  QueryWs q;
  if (!query_ws(P, s, q)) return CDX_ELAUNCH;
  if (workspace_bytes < q.bytes) return CDX_EINVAL;
  return mesh_order(points, P, static_cast<char*>(workspace), q, s) ? CDX_OK : CDX_ELAUNCH;
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
