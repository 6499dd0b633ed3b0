// Stream-level launchers of the GPIS std path shared by cdx_gpis_std and the closure
// (defined in cdx_gpis.hip).  ws buffers are caller-owned, sized by the *_ws_bytes helpers.
#pragma once
#include <hip/hip_runtime.h>

#include "cdx.h"

namespace cdx {
size_t gpis_var_ws_bytes(const cdx_gpis& g, int64_t M);
size_t gpis_grad_ws_bytes(const cdx_gpis& g, int64_t M);
// std[m] = sqrt|k0 − ‖L⁻¹k(x_m)‖²|, var_out[m] = the signed k0 − ‖L⁻¹k‖² (nullable).
int gpis_var_launch(const cdx_gpis& g, const double* X, int64_t M, double* std_out, double* var_out, void* ws,
                    hipStream_t s);
// gstd[sel[m]] = ∇std at X[m] (sel null: identity), scaled by var[sel[m]] from gpis_var_launch.
int gpis_grad_launch(const cdx_gpis& g, const double* X, int64_t M, const int64_t* sel, const double* var,
                     double* gstd, void* ws, hipStream_t s);
}  // namespace cdx
