// Sustained v_mfma_f64_16x16x4_f64 rate in the std GEMM's register shape: each wave owns a 4×4
// grid of 16×16 accumulators and issues 16 independent MFMAs per 4-deep substep (outer product of
// 4 A and 4 B fragments), 1, 2 or 4 waves per SIMD, no LDS, no barriers.  Bounds what the
// whitened std pass can reach on the 16x16x4 shape (the older mfma_f64_peak.hip chains 2–8
// accumulators per wave, a dependency-limited pattern).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/mfma_f64_tile.hip -o tools/microbench/mfma_f64_tile
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double dbl4 __attribute__((ext_vector_type(4)));

template <bool ROTATE>
__global__ __launch_bounds__(512) void tile(double* out, int iters, double seed) {
  __shared__ double pin[12288];  // 96 KB: one workgroup per CU
  pin[threadIdx.x] = seed;
  dbl4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0, 0, 0, 0};
  double a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { a[i] = seed + threadIdx.x * 1e-3 + i; b[i] = seed - threadIdx.x * 1e-3 - i; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    if (ROTATE) {  // new operands every substep (8 f64 VALU ops per 16 MFMAs)
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = a[i] * 0.999 + 1e-3; b[i] = b[i] * 1.001 - 1e-3; }
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 12345.678) out[0] = s + pin[threadIdx.x ^ 1];
}

// Operands from LDS as in the std kernel: per 4-deep substep 8 ds_read_b64 (4 A + 4 B fragments,
// rows padded to 144 doubles), register double buffer, no barriers (read-only LDS).
// mode 3: + the std kernel's per-K-step stage writes (4 ds_write_b64 K* + 4 ds_write_b128 B per
// thread, into a second buffer); mode 4: + its B-tile global loads (4 × 16 B per thread from a
// 32 MB operand, issued at the top of the step, consumed by the stage writes).
typedef double dbl2v __attribute__((ext_vector_type(2)));
template <int LDS_MODE>
__global__ __launch_bounds__(512) void tile_lds(double* out, int iters, double seed, const double* __restrict__ Bg) {
  __shared__ __attribute__((aligned(16))) double sm[2 * (16 * 144 + 16 * 272)];
  for (int i = threadIdx.x; i < 2 * (16 * 144 + 16 * 272); i += blockDim.x) sm[i] = seed + i * 1e-6;
  const int tid = threadIdx.x, ar = tid / 32, ac = (tid % 32) * 2, gm = tid & 127, gk = (tid >> 7) * 4;
  double* Kw = sm + 16 * 144 + 16 * 272;
  double* Aw = Kw + 16 * 144;
  dbl2v av[4];
  double kv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { av[i] = dbl2v{seed, seed + i}; kv[i] = seed * i; }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = (wave >> 2) * 64, wc = (wave & 3) * 64;
  const double* Kt = sm;
  const double* As = sm + 16 * 144;
  dbl4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0, 0, 0, 0};
  double fa[2][4], fb[2][4];
  auto frag = [&](int kk, double* a, double* b) {
    const int kra = (kk + (lane >> 4)) * 144 + (lane & 15);
    const int krb = (kk + (lane >> 4)) * 272 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = Kt[kra + wr + 16 * i]; b[i] = As[krb + wc + 16 * i]; }
  };
  frag(0, fa[0], fb[0]);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int kk = 0; kk < 16; kk += 4) {
      const int cur = (kk >> 2) & 1;
      frag((kk + 4) & 15, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0);
      if (LDS_MODE == 1) {
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
      }
    }
    if (LDS_MODE >= 3) {
      if (LDS_MODE >= 4) {
        const dbl2v* src = reinterpret_cast<const dbl2v*>(Bg + (int64_t)(((it * 16) & 2047) + ar) * 2048 +
                                                          ((blockIdx.x & 7) * 256) + ac);
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = src[i * 32];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) Kw[(gk + i) * 144 + gm] = kv[i];
      dbl2v* dst = reinterpret_cast<dbl2v*>(Aw + ar * 272 + ac);
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i * 32] = av[i];
    }
    if (LDS_MODE >= 2) __syncthreads();  // + one barrier per 16-deep K-step
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 12345.678) out[0] = s + Kw[tid] + Aw[tid];
}

template <int LDS_MODE>
void run_lds() {
  static double* Bg = nullptr;
  if (!Bg) {
    (void)hipMalloc(&Bg, 2048 * 2048 * 8);
    (void)hipMemset(Bg, 0, 2048 * 2048 * 8);
  }
  double* d;
  (void)hipMalloc(&d, 8);
  const int iters = 500, blocks = 256, threads = 512;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(tile_lds<LDS_MODE>, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0, Bg);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(tile_lds<LDS_MODE>, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0, Bg);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 5.0 * blocks * 8 * (double)iters * 64 * 2048.0;
  printf("{\"shape\": \"16x16x4 4x4 tile, LDS operands\", \"mode\": %d, \"waves_per_simd\": 2, \"ms\": %.3f, "
         "\"TFLOPs\": %.2f}\n", LDS_MODE, ms, flops / (ms * 1e-3) / 1e12);
  (void)hipFree(d);
}

template <bool ROTATE>
void run(int threads) {
  double* d;
  (void)hipMalloc(&d, 8);
  const int iters = 2000, blocks = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(tile<ROTATE>, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(tile<ROTATE>, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 5.0 * blocks * (threads / 64) * (double)iters * 16 * 2048.0;
  printf("{\"shape\": \"16x16x4 4x4 tile\", \"rotate\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"TFLOPs\": %.2f}\n",
         (int)ROTATE, threads / 256, ms, flops / (ms * 1e-3) / 1e12);
  (void)hipFree(d);
}

int main() {
  run<false>(256); run<false>(512); run<true>(256); run<true>(512);
  run_lds<0>(); run_lds<1>(); run_lds<2>(); run_lds<3>(); run_lds<4>();
  return 0;
}
