// Surviving-grasp record pack for the multi-GPU exchange (distributed.py).
//
// After an optimise loop every rank packs the candidates whose best-iterate margins are all
// positive — the reference's success test `opt_margin > 0` (optimize_pregrasp.py:226, :319, :405,
// :510, :611) — into a fixed-capacity float64 buffer that one all_gather exchanges (RCCL has no
// all-gatherv).  Row 0 is the header [stored, survived, capacity, 0, …]; rows 1.. are the
// survivors in candidate order:
//   [object_id, rank, candidate_id, best_loss, 1, margin[T], q[D], comp[T], target[3T], palm[6]]
// No host synchronisation: the buffer is zeroed (hipMemsetAsync: rows past the stored count stay
// zero, so the buffer is a pure function of the inputs), then one workgroup — thread t owns the
// contiguous candidates [t·C, t·C + C), C = ceil(E/1024) — scans the per-thread survivor counts and
// writes each survivor's row and the header.
#include <hip/hip_runtime.h>

#include "cdx.h"

namespace {

constexpr int PACK_THREADS = 1024;

__global__ __launch_bounds__(PACK_THREADS) void pack_survivors_kernel(
    int64_t E, int T, int D, const double* __restrict__ margin, const double* __restrict__ best_loss,
    const double* __restrict__ q, const double* __restrict__ comp, const double* __restrict__ target,
    const double* __restrict__ palm, double object_id, double rank, int64_t cand_offset, int64_t capacity,
    double* __restrict__ buf) {
  __shared__ int64_t wsum[PACK_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int W = 5 + T + D + T + 3 * T + 6;
  const int64_t C = (E + PACK_THREADS - 1) / PACK_THREADS;
  const int64_t e0 = (int64_t)t * C, e1 = e0 + C < E ? e0 + C : E;
  auto survives = [&](int64_t e) {
    bool ok = true;
    for (int f = 0; f < T; ++f) ok = ok && margin[e * T + f] > 0.0;  // NaN margins do not survive
    return ok;
  };
  int64_t n = 0;
  for (int64_t e = e0; e < e1; ++e) n += survives(e);
  int64_t inc = n;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t v = __shfl_up(inc, d);
    if (lane >= d) inc += v;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  int64_t before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < PACK_THREADS / 64; ++w) {
    before += w < wave ? wsum[w] : 0;
    total += wsum[w];
  }
  int64_t r = before + inc - n;  // survivors before this thread's first candidate
  for (int64_t e = e0; e < e1 && r < capacity; ++e) {
    if (!survives(e)) continue;
    double* o = buf + (r + 1) * W;
    o[0] = object_id;
    o[1] = rank;
    o[2] = (double)(e + cand_offset);
    o[3] = best_loss[e];
    o[4] = 1.0;
    int c = 5;
    for (int f = 0; f < T; ++f) o[c++] = margin[e * T + f];
    for (int i = 0; i < D; ++i) o[c++] = q[e * D + i];
    for (int f = 0; f < T; ++f) o[c++] = comp[e * T + f];
    for (int i = 0; i < 3 * T; ++i) o[c++] = target[e * 3 * T + i];
    for (int i = 0; i < 6; ++i) o[c++] = palm[e * 6 + i];
    ++r;
  }
  if (t == 0) {
    buf[0] = (double)(total < capacity ? total : capacity);
    buf[1] = (double)total;
    buf[2] = (double)capacity;
  }
}

}  // namespace

extern "C" int cdx_pack_survivors(int64_t E, int32_t n_tips, int32_t n_dofs, const double* margin,
                                  const double* best_loss, const double* q, const double* comp, const double* target,
                                  const double* palm, double object_id, double rank, int64_t cand_offset,
                                  int64_t capacity, double* buf, cdx_stream_t stream) {
  if (E < 0 || capacity < 0 || n_tips < 1 || n_tips > CDX_MAX_TIPS || n_dofs < 0 || n_dofs > CDX_MAX_DOFS || !buf)
    return CDX_EINVAL;
  if (E > 0 && (!margin || !best_loss || !q || !comp || !target || !palm)) return CDX_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int W = 5 + n_tips + n_dofs + n_tips + 3 * n_tips + 6;
  if (hipMemsetAsync(buf, 0, (size_t)(capacity + 1) * W * sizeof(double), s) != hipSuccess) return CDX_ELAUNCH;
  hipLaunchKernelGGL(pack_survivors_kernel, dim3(1), dim3(PACK_THREADS), 0, s, E,
                     (int)n_tips, (int)n_dofs, margin, best_loss, q, comp, target, palm, object_id, rank, cand_offset,
                     capacity, buf);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}
