// Host/device qualifiers and tiny fixed-size linear algebra shared by the HIP kernels
// and by the host build used in CPU tests (libcdx_host.so: the SAME per-candidate code,
// compiled for x86 so the analytic backward can be checked against the oracle without
// a GPU).  Not a portability layer: device code is gfx950-only.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CDX_HD __host__ __device__ __forceinline__
#define CDX_HDM __host__ __device__ __forceinline__  // member functions
#else
#define CDX_HD static inline
#define CDX_HDM inline
#endif

#include "../../include/cdx.h"

namespace cdx {

template <typename T>
CDX_HD void mat3_mul(const T* a, const T* b, T* c) {  // c = a·b (row-major 3×3)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) c[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
template <typename T>
CDX_HD void mat3_mul_tn(const T* a, const T* b, T* c) {  // c = aᵀ·b
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) c[3 * i + j] = a[i] * b[j] + a[3 + i] * b[3 + j] + a[6 + i] * b[6 + j];
}
template <typename T>
CDX_HD void mat3_mul_nt(const T* a, const T* b, T* c) {  // c = a·bᵀ
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) c[3 * i + j] = a[3 * i] * b[3 * j] + a[3 * i + 1] * b[3 * j + 1] + a[3 * i + 2] * b[3 * j + 2];
}
template <typename T>
CDX_HD void mat3_vec(const T* a, const T* v, T* out) {  // out = a·v
  for (int i = 0; i < 3; ++i) out[i] = a[3 * i] * v[0] + a[3 * i + 1] * v[1] + a[3 * i + 2] * v[2];
}
template <typename T>
CDX_HD void mat3t_vec(const T* a, const T* v, T* out) {  // out = aᵀ·v
  for (int i = 0; i < 3; ++i) out[i] = a[i] * v[0] + a[3 + i] * v[1] + a[6 + i] * v[2];
}
template <typename T>
CDX_HD T dot3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// float32 sin/cos of the joint angles.  The device rounds the f64 result (correctly rounded f32
// except on double-rounding ties), as the host's glibc sinf/cosf and the reference's CPU torch
// ops are: the collision cost's 1/d near contact turns one ulp of an f32 FK anchor into 1e-4.
#if defined(__HIP_DEVICE_COMPILE__)
CDX_HD float cdx_sinf(float x) { return (float)sin((double)x); }
CDX_HD float cdx_cosf(float x) { return (float)cos((double)x); }
#else
CDX_HD float cdx_sinf(float x) { return sinf(x); }
CDX_HD float cdx_cosf(float x) { return cosf(x); }
#endif

}  // namespace cdx
