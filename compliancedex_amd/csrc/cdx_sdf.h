// Point → triangle closest point (float32), shared by the gfx950 kernel and the host
// build.  Follows the Voronoi-region test order of the reference TorchSDF kernel
// (thirdparty/TorchSDF/torchsdf/csrc/unbatched_triangle_distance_cuda.cu:132-174 helpers,
// :201-237 per-face body).  Compiled with FP contraction OFF and 1/sqrt correctly rounded so
// the device result is bit-identical to the CPU oracle (the reference's CUDA rsqrt is a
// ≤2-ulp approximation and not reproducible on other hardware).
#pragma once
#include "cdx_hd.h"

#pragma clang fp contract(off)

namespace cdx {

struct F3 { float x, y, z; };
CDX_HD F3 f3(float x, float y, float z) { F3 r; r.x = x; r.y = y; r.z = z; return r; }
CDX_HD F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
CDX_HD F3 add(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
CDX_HD F3 scl(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
CDX_HD float dotf(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
CDX_HD F3 crossf(F3 a, F3 b) { return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
CDX_HD float rsqrt_cr(float x) { return 1.0f / sqrtf(x); }

// Distance of p to one face; returns squared distance, writes closest point, unit
// (p − c) direction and the ±1 side of the (v1−v2)×(v1−v3) face normal.
CDX_HD float point_face(F3 p, F3 v1, F3 v2, F3 v3, F3& clst, F3& nrm, int& sgn) {
  const F3 e12 = sub(v2, v1), e23 = sub(v3, v2), e31 = sub(v1, v3);
  const F3 normal = crossf(sub(v1, v2), e31);
  const float uab = dotf(sub(p, v1), e12) / dotf(e12, e12);
  const float uca = dotf(sub(p, v3), e31) / dotf(e31, e31);
  F3 c;
  if (uca > 1 && uab < 0) {
    c = v1;
  } else {
    const float ubc = dotf(sub(p, v2), e23) / dotf(e23, e23);
    if (uab > 1 && ubc < 0) {
      c = v2;
    } else if (ubc > 1 && uca < 0) {
      c = v3;
    } else if (uab <= 1 && uab >= 0 && dotf(crossf(normal, e12), sub(p, v1)) <= 0) {
      c = add(v1, scl(e12, uab));
    } else if (ubc <= 1 && ubc >= 0 && dotf(crossf(normal, e23), sub(p, v2)) <= 0) {
      c = add(v2, scl(e23, ubc));
    } else if (uca <= 1 && uca >= 0 && dotf(crossf(normal, e31), sub(p, v3)) <= 0) {
      c = add(v3, scl(e31, uca));
    } else {
      const float inv_len = rsqrt_cr(dotf(normal, normal));
      const F3 un = scl(normal, inv_len);
      const float d = (p.x - v1.x) * un.x + (p.y - v1.y) * un.y + (p.z - v1.z) * un.z;
      c = sub(p, scl(un, d));
    }
  }
  const F3 dv = sub(p, c);
  const float dd = dotf(dv, dv);
  nrm = scl(dv, rsqrt_cr(1e-16f + dd));
  sgn = dotf(dv, normal) >= 0 ? 1 : -1;
  clst = c;
  return dd;
}

// ---------------------------------------------------------------- double dispatch
// The reference dispatches float AND double (AT_DISPATCH_FLOATING_TYPES, .cu:282); with double inputs
// its per-face body (.cu:201-237) computes in double EXCEPT where it names float: the edge parameter
// passed to point_at is a `float t` (.cu:171-173: c = v + e·(double)(float)u), and the squared
// distance is stored through `float dist` (.cu:237) — so the result's distance is a float value, and
// the tile comparisons (.cu:238, :245) compare float values widened to double.  The 1e-16f of the
// normal's rsqrt is a float literal widened to double.  rsqrt is correctly rounded 1/sqrt here too.
struct D3 { double x, y, z; };
CDX_HD D3 d3(double x, double y, double z) { D3 r; r.x = x; r.y = y; r.z = z; return r; }
CDX_HD D3 subd(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
CDX_HD D3 addd(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
CDX_HD D3 scld(D3 a, double s) { return d3(a.x * s, a.y * s, a.z * s); }
CDX_HD double dotd(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
CDX_HD D3 crossd(D3 a, D3 b) { return d3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
CDX_HD double rsqrt_crd(double x) { return 1.0 / sqrt(x); }

CDX_HD float point_face_d(D3 p, D3 v1, D3 v2, D3 v3, D3& clst, D3& nrm, int& sgn) {
  const D3 e12 = subd(v2, v1), e23 = subd(v3, v2), e31 = subd(v1, v3);
  const D3 normal = crossd(subd(v1, v2), e31);
  const double uab = dotd(subd(p, v1), e12) / dotd(e12, e12);
  const double uca = dotd(subd(p, v3), e31) / dotd(e31, e31);
  D3 c;
  if (uca > 1 && uab < 0) {
    c = v1;
  } else {
    const double ubc = dotd(subd(p, v2), e23) / dotd(e23, e23);
    if (uab > 1 && ubc < 0) {
      c = v2;
    } else if (ubc > 1 && uca < 0) {
      c = v3;
    } else if (uab <= 1 && uab >= 0 && dotd(crossd(normal, e12), subd(p, v1)) <= 0) {
      c = addd(v1, scld(e12, (double)(float)uab));
    } else if (ubc <= 1 && ubc >= 0 && dotd(crossd(normal, e23), subd(p, v2)) <= 0) {
      c = addd(v2, scld(e23, (double)(float)ubc));
    } else if (uca <= 1 && uca >= 0 && dotd(crossd(normal, e31), subd(p, v3)) <= 0) {
      c = addd(v3, scld(e31, (double)(float)uca));
    } else {
      const double inv_len = rsqrt_crd(dotd(normal, normal));
      const D3 un = scld(normal, inv_len);
      const double d = (p.x - v1.x) * un.x + (p.y - v1.y) * un.y + (p.z - v1.z) * un.z;
      c = subd(p, scld(un, d));
    }
  }
  const D3 dv = subd(p, c);
  const double dd = dotd(dv, dv);
  nrm = scld(dv, rsqrt_crd((double)1e-16f + dd));
  sgn = dotd(dv, normal) >= 0 ? 1 : -1;
  clst = c;
  return (float)dd;
}

// The reference scans faces in 512-face tiles (.cu:186-246): inside a tile the first
// face is always taken and later faces replace it only when strictly closer (:238);
// a tile's winner replaces the running result only when strictly closer (:245), except
// that tile 0's winner is always taken.  With NaN distances (degenerate faces) this is
// not a plain argmin, so every implementation keeps this exact rule.
#define CDX_SDF_REF_TILE 512

// ---------------------------------------------------------------- culled path
// Per-face quantities of point_face, computed once per face with the SAME IEEE operations
// (FP contraction off), so face_dist2 below returns bit-for-bit the squared distance
// point_face returns.  40 floats: one s_load_dwordx8 ×5 per face on the device.
// The padding words hold the face's own bounding sphere (centre bx..bz = the vertices' mean, radius br, |centre|
// bn) for the culled kernel's per-face bound (the same bound as a chunk's sphere, face by face).
struct FaceRec {
  F3 v1; int idx;  F3 v2; float den12;  F3 v3; float den23;  F3 e12; float den31;
  F3 e23; float bx;  F3 e31; float by;  F3 ne12; float bz;  F3 ne23; float br;
  F3 ne31; float bn;  F3 un; float kappa;   // kappa = |e12||e31| / |n| (conditioning, 1/sinθ)
};

CDX_HD FaceRec face_rec(F3 v1, F3 v2, F3 v3, int idx) {
  FaceRec r;
  r.v1 = v1; r.v2 = v2; r.v3 = v3; r.idx = idx;
  r.e12 = sub(v2, v1); r.e23 = sub(v3, v2); r.e31 = sub(v1, v3);
  const F3 normal = crossf(sub(v1, v2), r.e31);
  r.den12 = dotf(r.e12, r.e12); r.den23 = dotf(r.e23, r.e23); r.den31 = dotf(r.e31, r.e31);
  r.ne12 = crossf(normal, r.e12); r.ne23 = crossf(normal, r.e23); r.ne31 = crossf(normal, r.e31);
  const float nn = dotf(normal, normal);
  r.un = scl(normal, rsqrt_cr(nn));
  r.kappa = sqrtf(r.den12) * sqrtf(r.den31) / sqrtf(nn);
  const float third = 1.f / 3.f;
  r.bx = (v1.x + v2.x + v3.x) * third;
  r.by = (v1.y + v2.y + v3.y) * third;
  r.bz = (v1.z + v2.z + v3.z) * third;
  const F3 c = f3(r.bx, r.by, r.bz);
  r.br = fmaxf(fmaxf(sqrtf(dotf(sub(v1, c), sub(v1, c))), sqrtf(dotf(sub(v2, c), sub(v2, c)))),
               sqrtf(dotf(sub(v3, c), sub(v3, c)))) * (1.f + 1e-5f);
  r.bn = sqrtf(r.bx * r.bx + r.by * r.by + r.bz * r.bz);
  return r;
}

// A face whose point_face can produce NaN/inf for a finite point of magnitude ≤ 1e4
// (zero-length edge, zero normal, non-finite or huge vertex).  Meshes holding one take
// the exact tile-rule path, where NaN distances have the reference's semantics.
CDX_HD bool face_may_nan(const FaceRec& r) {
  const float lim = 1e4f;
  const bool fin = fabsf(r.v1.x) <= lim && fabsf(r.v1.y) <= lim && fabsf(r.v1.z) <= lim &&
                   fabsf(r.v2.x) <= lim && fabsf(r.v2.y) <= lim && fabsf(r.v2.z) <= lim &&
                   fabsf(r.v3.x) <= lim && fabsf(r.v3.y) <= lim && fabsf(r.v3.z) <= lim;
  const float nn = dotf(crossf(sub(r.v1, r.v2), r.e31), crossf(sub(r.v1, r.v2), r.e31));
  return !(fin && r.den12 > 1e-20f && r.den23 > 1e-20f && r.den31 > 1e-20f && nn > 1e-30f);
}

// Squared distance of point_face from the precomputed record (same branch order).
CDX_HD float face_dist2(F3 p, const FaceRec& r) {
  const F3 w1 = sub(p, r.v1);
  const float uab = dotf(w1, r.e12) / r.den12;
  const F3 w3 = sub(p, r.v3);
  const float uca = dotf(w3, r.e31) / r.den31;
  const F3 w2 = sub(p, r.v2);
  const float ubc = dotf(w2, r.e23) / r.den23;
  F3 c;
  if (uca > 1 && uab < 0) {
    c = r.v1;
  } else if (uab > 1 && ubc < 0) {
    c = r.v2;
  } else if (ubc > 1 && uca < 0) {
    c = r.v3;
  } else if (uab <= 1 && uab >= 0 && dotf(r.ne12, w1) <= 0) {
    c = add(r.v1, scl(r.e12, uab));
  } else if (ubc <= 1 && ubc >= 0 && dotf(r.ne23, w2) <= 0) {
    c = add(r.v2, scl(r.e23, ubc));
  } else if (uca <= 1 && uca >= 0 && dotf(r.ne31, w3) <= 0) {
    c = add(r.v3, scl(r.e31, uca));
  } else {
    const float d = w1.x * r.un.x + w1.y * r.un.y + w1.z * r.un.z;
    c = sub(p, scl(r.un, d));
  }
  const F3 dv = sub(p, c);
  return dotf(dv, dv);
}

}  // namespace cdx
