// GPIS covariance functions (gpis.py:16-29) evaluated from a squared distance.
//   k    : covariance k(x, x_j)
//   kd   : ∂k/∂x = kd·(x − x_j)   (the autograd gradient through cdist: _cdist_backward
//          gives (x − x_j)/r, times dk/dr; TPS dk/dr = 6r² − 6Rr ⇒ kd = 6r − 6R)
//   k0   : k(x, x), the prior variance the posterior std subtracts from (gpis.py:57)
#pragma once
#include "cdx_hd.h"

namespace cdx {

template <int KT>
CDX_HD void gpis_k(double r2, double R, double inv_s2, double& k, double& kd) {
  if (KT == CDX_KERNEL_TPS) {
    const double r = sqrt(r2);
    k = 2.0 * (r2 * r) - 3.0 * R * r2 + R * R * R;
    kd = 6.0 * r - 6.0 * R;
  } else if (KT == CDX_KERNEL_RBF) {
    k = exp(-0.5 * r2 * inv_s2);
    kd = -k * inv_s2;
  } else {
    const double r = sqrt(r2);
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
