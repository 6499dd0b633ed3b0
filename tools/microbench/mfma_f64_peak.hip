// Measures the sustained v_mfma_f64_16x16x4_f64 rate on every CU (operands in registers,
// independent accumulators) — the ceiling the GPIS std GEMM is priced against.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void peak(double* out, int iters, double seed, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  dbl4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = dbl4{0, 0, 0, 0};
  double a[NACC], b[NACC];
  for (int i = 0; i < NACC; ++i) { a[i] = seed + threadIdx.x * 1e-3 + i; b[i] = seed - threadIdx.x * 1e-3 - i; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[i], acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[0] = s;
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int NACC>
__global__ __launch_bounds__(256) void peak4(double* out, int iters, double seed) {
  double acc[NACC];
  double a[NACC], b[NACC];
  for (int i = 0; i < NACC; ++i) { acc[i] = 0; a[i] = seed + threadIdx.x * 1e-3 + i; b[i] = seed - threadIdx.x * 1e-3 - i; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[i], b[i], acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;
}

template <int NACC>
void run4(int blocks_per_cu) {
  double* d;
  (void)hipMalloc(&d, 8);
  const int iters = 8000, blocks = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(peak4<NACC>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(peak4<NACC>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 5.0 * blocks * 4.0 * iters * NACC * 512.0;  // 4 blocks of 4x4x4 per instruction
  printf("{\"shape\": \"4x4x4_4b\", \"nacc\": %d, \"blocks_per_cu\": %d, \"ms\": %.3f, \"TFLOPs\": %.2f}\n", NACC,
         blocks_per_cu, ms, flops / (ms * 1e-3) / 1e12);
}

template <int NACC>
void run(int blocks_per_cu) {
  double* d;
  (void)hipMalloc(&d, 8);
  unsigned long long* clk;
  (void)hipMallocManaged(&clk, 16);
  const int iters = 4000;
  const int blocks = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(peak<NACC>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0, clk);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(peak<NACC>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0, clk);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 5.0 * blocks * 4.0 /*waves*/ * iters * NACC * 2048.0;
  (void)hipDeviceSynchronize();
  const double ghz = (double)clk[0] / (double)clk[1] * 0.1;  // s_memrealtime ticks at 100 MHz
  const double cyc_per_mfma = (double)clk[0] / ((double)iters * NACC) * (blocks_per_cu * 4 / 4.0);
  printf("{\"nacc\": %d, \"blocks_per_cu\": %d, \"ms\": %.3f, \"TFLOPs\": %.2f, \"clock_GHz\": %.3f, "
         "\"cycles_per_mfma_per_simd\": %.1f}\n", NACC, blocks_per_cu, ms, flops / (ms * 1e-3) / 1e12, ghz, cyc_per_mfma);
  (void)hipFree(d);
}

int main() {
  run<2>(1); run<4>(1); run<8>(1); run<2>(2); run<4>(2); run<8>(2); run<2>(4); run<4>(4); run<8>(4); run<4>(8);
  run4<8>(1); run4<8>(2); run4<16>(2); run4<8>(4);
  return 0;
}
