// Stream-level launchers of the GPIS std path shared by cdx_gpis_std and the closure
// (defined in cdx_gpis.hip).  ws buffers are caller-owned, sized by the *_ws_bytes helpers.
#pragma once
#include <hip/hip_runtime.h>

#include "cdx.h"

namespace cdx {
size_t gpis_var_ws_bytes(const cdx_gpis& g, int64_t M);
size_t gpis_grad_ws_bytes(const cdx_gpis& g, int64_t M);
// Bytes of the stored whitened vectors V = (L⁻¹K*ᵀ)ᵀ of M queries ([round_up(M, 128), N_pad] f64).
size_t gpis_v_bytes(const cdx_gpis& g, int64_t M);
// Per-group argmax selection fused into the std finalize: rows [t·T, t·T + T) form group t; sel[t]
// = the row of the first maximum of log(100·std) in the group (optimize_pregrasp.py:730's max),
// Xg[t] = X[sel[t]].
struct VarSelect {
  int T;
  int64_t* sel;
  double* Xg;
};
// std[m] = sqrt|k0 − ‖L⁻¹k(x_m)‖²|, var_out[m] = the signed k0 − ‖L⁻¹k‖² (nullable); vout
// (nullable, gpis_v_bytes) receives V; vs (nullable; M a multiple of vs->T) selects per group.
int gpis_var_launch(const cdx_gpis& g, const double* X, int64_t M, double* std_out, double* var_out, void* ws,
                    hipStream_t s, double* vout = nullptr, const VarSelect* vs = nullptr);
// gstd[sel[m]] = ∇std at X[m] (sel null: identity), scaled by var[sel[m]] from gpis_var_launch.
// vin null: W = E11⁻¹k (2N² flops per query); vin = the V of gpis_var_launch: W = L⁻ᵀ v from row
// sel[m] of V (N² flops per query; needs g.Linv).
// vrow (nullable): the V row of query m is vrow[m] instead of sel[m] (the refine pass's list positions).
int gpis_grad_launch(const cdx_gpis& g, const double* X, int64_t M, const int64_t* sel, const double* var,
                     double* gstd, void* ws, hipStream_t s, const double* vin = nullptr,
                     const int64_t* vrow = nullptr);
// Refine pass behind the split-precision screen: the whitened fp64 pass (V = K*·L⁻ᵀ, Σ V²) for the
// rows rows[0 .. G + *extra) of X (device-side count, at most Mcap), cut into equal pieces (one per
// CU) whatever the count; V rows go to vout at the list positions ([round_up(Mcap, 128), N_pad]),
// Σ V² per (stripe, position) to the returned partial [N_pad/256][*M_pad_out].
size_t gpis_refine_ws_bytes(const cdx_gpis& g, int64_t Mcap);
// Zeroes the refine workspace's cut-unit arrival counters (once after allocation; every launch
// leaves them zero).
int gpis_refine_reset(const cdx_gpis& g, int64_t Mcap, void* ws, hipStream_t s);
int gpis_refine_launch(const cdx_gpis& g, const double* X, const int* rows, const int* extra, int G, int64_t Mcap,
                       void* ws, double* vout, hipStream_t s, double** partial_out, int64_t* M_pad_out);
}  // namespace cdx
