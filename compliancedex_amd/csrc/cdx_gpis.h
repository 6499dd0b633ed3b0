// GPIS covariance functions (gpis.py:16-29) evaluated from a squared distance.
//   k    : covariance k(x, x_j)
//   kd   : ∂k/∂x = kd·(x − x_j)   (the autograd gradient through cdist: _cdist_backward
//          gives (x − x_j)/r, times dk/dr; TPS dk/dr = 6r² − 6Rr ⇒ kd = 6r − 6R)
//   k0   : k(x, x), the prior variance the posterior std subtracts from (gpis.py:57)
#pragma once
#include "cdx_hd.h"

namespace cdx {

// sqrt of a non-negative squared distance.  Device: v_rsq_f64 + one Goldschmidt step + two
// Newton corrections (the core of the compiler's sqrt without its denormal/inf scaling, which
// a clamped r² ≥ 1e-200 never needs); r² = 0 returns 1e-100, harmless in every use here
// (k(1e-100) = k(0) to 1e-200, and ∂k/∂x carries a factor (x − x_j) = 0).
CDX_HD double sqrt_r2(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(CDX_FAST_SQRT)
  x = fmax(x, 1e-200);
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double e = fma(-h, g, 0.5);
  g = fma(g, e, g);
  h = fma(h, e, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
#else
  return sqrt(x);
#endif
}

// sqrt_r2 without its final Newton correction (≤ 1 ulp from the rounded root): the whitened
// pass's on-chip K* generation (CDX_GEN_SQRT_FULL keeps the full sequence there).
CDX_HD double sqrt_r2_f32seed(double x);
CDX_HD double sqrt_r2_gen(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(CDX_GEN_RSQ32)  // A/B: the f32-seeded root (≈ 2⁻⁴⁵) in K* too
  return sqrt_r2_f32seed(x);
#elif defined(__HIP_DEVICE_COMPILE__) && defined(CDX_FAST_SQRT) && !defined(CDX_GEN_SQRT_FULL)
  x = fmax(x, 1e-200);
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double e = fma(-h, g, 0.5);
  g = fma(g, e, g);
  h = fma(h, e, h);
  const double d = fma(-g, g, x);
  return fma(d, h, g);
#else
  return sqrt_r2(x);
#endif
}

// sqrt(x) from an f32 reciprocal-root seed and one f64 Newton step (relative error ≈ 2⁻⁴⁵, 1e-14; against
// ≤ 1 ulp for sqrt_r2_gen): the f32 transcendental and the two conversions replace v_rsq_f64 and the
// Goldschmidt refinement — the GPIS mean's per-pair root (CDX_MEAN_RSQ32 builds).
CDX_HD double sqrt_r2_f32seed(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float xf = fmaxf((float)x, 1e-30f);
  const double y = (double)__builtin_amdgcn_rsqf(xf);
  const double g = x * y, h = 0.5 * y;
  const double d = fma(-g, g, x);
  return fma(d, h, g);
#else
  return sqrt(x);
#endif
}

template <int KT, bool GENSQRT = false>
CDX_HD void gpis_k(double r2, double R, double inv_s2, double& k, double& kd) {
  if (KT == CDX_KERNEL_TPS) {
    const double r = GENSQRT ? sqrt_r2_gen(r2) : sqrt_r2(r2);
    k = 2.0 * (r2 * r) - 3.0 * R * r2 + R * R * R;
    kd = 6.0 * r - 6.0 * R;
  } else if (KT == CDX_KERNEL_RBF) {
    k = exp(-0.5 * r2 * inv_s2);
    kd = -k * inv_s2;
  } else {
    const double r = GENSQRT ? sqrt_r2_gen(r2) : sqrt_r2(r2);
    const double kr = exp(-0.5 * r2 * inv_s2);
    k = 0.3 * kr + 0.7 * (2.0 * (r2 * r) - 3.0 * R * r2 + R * R * R);
    kd = 0.3 * (-kr * inv_s2) + 0.7 * (6.0 * r - 6.0 * R);
  }
}

template <int KT>
CDX_HD double gpis_k0(double R) {
  if (KT == CDX_KERNEL_TPS) return R * R * R;
  if (KT == CDX_KERNEL_RBF) return 1.0;
  return 0.3 + 0.7 * (R * R * R);
}

}  // namespace cdx
