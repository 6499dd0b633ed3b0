// Surviving-grasp record pack for the multi-GPU exchange (distributed.py).
//
// After an optimise loop every rank packs the candidates whose best-iterate margins are all
// positive — the reference's success test `opt_margin > 0` (optimize_pregrasp.py:226, :319, :405,
// :510, :611) — into a fixed-capacity float64 buffer that one all_gather exchanges (RCCL has no
// all-gatherv).  Row 0 is the header [stored, survived, capacity, 0, …]; rows 1.. are the
// survivors in candidate order:
//   [object_id, rank, candidate_id, best_loss, 1, margin[T], q[D], comp[T], target[3T], palm[6]]
// No host synchronisation and no memset: one workgroup walks the candidates in tiles of 1024 (one
// candidate per thread): a block scan of the tile's survival flags gives each survivor its row and
// an LDS list (row → candidate); then all threads write the tile's rows element by element (row-major,
// consecutive threads on consecutive doubles: coalesced stores, four independent gathers in flight
// per thread).  Finally the
// rows past the stored count are zeroed, so the buffer is a pure function of the inputs, and thread 0
// writes the header.  (The first version — thread t packing its own C = ⌈E/1024⌉ candidates row by
// row after a memset — took ≈ 0.1 ms at E = 4096: each thread's 47-field rows were serial,
// uncoalesced stores.)
#include <hip/hip_runtime.h>

#include "cdx.h"

namespace {

constexpr int PACK_THREADS = 1024;

__global__ __launch_bounds__(PACK_THREADS) void pack_survivors_kernel(
    int64_t E, int T, int D, const double* __restrict__ margin, const double* __restrict__ best_loss,
    const double* __restrict__ q, const double* __restrict__ comp, const double* __restrict__ target,
    const double* __restrict__ palm, double object_id, double rank, int64_t cand_offset, int64_t capacity,
    double* __restrict__ buf) {
  __shared__ int wsum[PACK_THREADS / 64];
  __shared__ int list[PACK_THREADS];  // tile-local row → candidate offset in the tile
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int W = 5 + T + D + T + 3 * T + 6;
  // field c of a record for candidate e: a branch-free address (selects, no divergent loads), so that
  // the unrolled element loop below keeps several gathers in flight per thread
  auto field = [&](int64_t e, int c) -> double {
    int o = c - 5;
    const double* p = margin + e * T + (o < 0 ? 0 : o);
    o -= T;
    p = o >= 0 ? q + e * D + o : p;
    o -= D;
    p = o >= 0 ? comp + e * T + o : p;
    o -= T;
    p = o >= 0 ? target + e * 3 * T + o : p;
    o -= 3 * T;
    p = o >= 0 ? palm + e * 6 + o : p;
    const double v = *p;
    if (c >= 5) return v;
    const double h = c == 0 ? object_id : (c == 1 ? rank : (c == 2 ? (double)(e + cand_offset) : 1.0));
    return c == 3 ? best_loss[e] : h;
  };
  int64_t base = 0;  // survivors before this tile
  for (int64_t e0 = 0; e0 < E; e0 += PACK_THREADS) {
    const int64_t e = e0 + t;
    bool ok = e < E;
    for (int f = 0; ok && f < T; ++f) ok = margin[e * T + f] > 0.0;  // NaN margins do not survive
    // block scan of the flags: ballot prefix within the wave, wave totals through LDS
    const unsigned long long bal = __ballot(ok);
    const int inwave = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    int before = 0, tile_n = 0;
#pragma unroll
    for (int w = 0; w < PACK_THREADS / 64; ++w) {
      before += w < wave ? wsum[w] : 0;
      tile_n += wsum[w];
    }
    if (ok) list[before + inwave] = t;
    __syncthreads();
    // rows base + [0, tile_n) of which those below `capacity` are stored
    const int64_t n_store = base >= capacity ? 0 : (capacity - base < tile_n ? capacity - base : tile_n);
    const int n_el = (int)n_store * W;  // ≤ 1024·W
    constexpr int U = 4;                 // elements per thread in flight
    for (int i0 = t; i0 < n_el; i0 += U * PACK_THREADS) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + u * PACK_THREADS, n_el - 1), r = i / W;
        v[u] = field(e0 + list[r], i - r * W);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (i0 + u * PACK_THREADS < n_el) buf[(base + 1) * W + i0 + u * PACK_THREADS] = v[u];
    }
    base += tile_n;
    __syncthreads();  // wsum / list reused by the next tile
  }
  const int64_t stored = base < capacity ? base : capacity;
  for (int64_t i = stored * W + t; i < capacity * W; i += PACK_THREADS) buf[W + i] = 0.0;  // unused rows
  for (int c = t; c < W; c += PACK_THREADS)
    buf[c] = c == 0 ? (double)stored : (c == 1 ? (double)base : (c == 2 ? (double)capacity : 0.0));
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
  hipLaunchKernelGGL(pack_survivors_kernel, dim3(1), dim3(PACK_THREADS), 0, s, E,
                     (int)n_tips, (int)n_dofs, margin, best_loss, q, comp, target, palm, object_id, rank, cand_offset,
                     capacity, buf);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}
