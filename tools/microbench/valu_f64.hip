// Sustained f64 VALU rates on every CU: v_fma_f64 with independent accumulators, and
// v_rsq_f64 — the instruction mix of the GPIS mean kernel and the K* generation.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NACC>
__global__ __launch_bounds__(256) void fma_rate(double* out, int iters, double seed) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = seed + threadIdx.x * 1e-3 + i;
  const double a = 1.0000001, b = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fma(acc[i], a, b);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void rsq_rate(double* out, int iters, double seed) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = seed + threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_rsq(acc[i]) + 1.0;
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;
}

template <typename K>
static void timeit(const char* name, K kern, int nacc, int per_iter_ops, int blocks_per_cu) {
  double* d;
  (void)hipMalloc(&d, 8);
  const int iters = 4000, blocks = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double lane_ops = 5.0 * blocks * 256.0 * iters * nacc * per_iter_ops;
  // lanes per cycle per CU at 2.4 GHz
  printf("{\"op\": \"%s\", \"nacc\": %d, \"blocks_per_cu\": %d, \"ms\": %.3f, \"Glane_ops\": %.1f, "
         "\"lanes_per_clk_per_cu\": %.2f}\n",
         name, nacc, blocks_per_cu, ms, lane_ops / (ms * 1e-3) / 1e9, lane_ops / (ms * 1e-3) / 2.4e9 / 256.0);
  (void)hipFree(d);
}

int main() {
  for (int bpc : {1, 4}) {
    timeit("v_fma_f64", fma_rate<4>, 4, 1, bpc);
    timeit("v_fma_f64", fma_rate<8>, 8, 1, bpc);
    timeit("v_fma_f64", fma_rate<16>, 16, 1, bpc);
    timeit("v_rsq_f64+add", rsq_rate<8>, 8, 1, bpc);
  }
  return 0;
}
