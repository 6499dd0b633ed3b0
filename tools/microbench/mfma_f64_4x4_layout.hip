// Probes the lane layout of v_mfma_f64_4x4x4_4b_f64: for every (A-lane, B-lane) pair, one-hot
// operands; prints which D lanes receive the product.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void probe(double* out) {
  const int la = blockIdx.x / 64, lb = blockIdx.x % 64, l = threadIdx.x;
  double a = l == la ? 1.0 : 0.0, b = l == lb ? 1.0 : 0.0;
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[blockIdx.x * 64 + l] = d;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 4096 * 64 * 8);
  hipLaunchKernelGGL(probe, dim3(4096), dim3(64), 0, 0, d);
  std::vector<double> h(4096 * 64);
  (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  for (int p = 0; p < 4096; ++p)
    for (int l = 0; l < 64; ++l)
      if (h[p * 64 + l] != 0.0) printf("%d %d %d %g\n", p / 64, p % 64, l, h[p * 64 + l]);
  return 0;
}
