// Surviving-grasp record pack for the multi-GPU exchange (distributed.py).
//
// After an optimise loop every rank packs the candidates whose best-iterate margins are all
// positive — the reference's success test `opt_margin > 0` (optimize_pregrasp.py:226, :319, :405,
// :510, :611) — into a fixed-capacity float64 buffer that one all_gather exchanges (RCCL has no
// all-gatherv).  Row 0 is the header [stored, survived, capacity, 0, …]; rows 1.. are the
// survivors in candidate order:
//   [object_id, rank, candidate_id, best_loss, 1, margin[T], q[D], comp[T], target[3T], palm[6]]
// No host synchronisation and no memset; two launches, both spread over the chip:
//   1. pack_count_kernel    one 64-candidate tile per wave: its survivor count (ballot);
//   2. pack_survivors_kernel one tile per 64-thread workgroup: the tile's first row = Σ of the earlier
//      tiles' counts (a workgroup reduction over the counts array), a ballot prefix gives each survivor
//      its row, then the tile's rows are written element by element (consecutive lanes on consecutive
//      doubles: coalesced stores, several gathers in flight per lane); rows past the stored count are
//      zeroed grid-stride, so the buffer is a pure function of the inputs; workgroup 0 writes the header.
// (Round 2's one-workgroup version walked the candidates in 1024-wide tiles: ≈ 0.1 ms at E = 4096,
// latency-bound on one CU.)
#include <hip/hip_runtime.h>

#include <mutex>

#include "cdx.h"

namespace {

constexpr int PACK_TILE = 64;  // candidates per tile = threads per workgroup (one wave)

__device__ __forceinline__ bool survives(int64_t e, int64_t E, int T, const double* __restrict__ margin) {
  bool ok = e < E;
  for (int f = 0; ok && f < T; ++f) ok = margin[e * T + f] > 0.0;  // NaN margins do not survive
  return ok;
}

__global__ __launch_bounds__(PACK_TILE) void pack_count_kernel(int64_t E, int T, const double* __restrict__ margin,
                                                               int* __restrict__ counts) {
  const int64_t e = (int64_t)blockIdx.x * PACK_TILE + threadIdx.x;
  const unsigned long long bal = __ballot(survives(e, E, T, margin));
  if (threadIdx.x == 0) counts[blockIdx.x] = __popcll(bal);
}

__global__ __launch_bounds__(PACK_TILE) void pack_survivors_kernel(
    int64_t E, int T, int D, const double* __restrict__ margin, const double* __restrict__ best_loss,
    const double* __restrict__ q, const double* __restrict__ comp, const double* __restrict__ target,
    const double* __restrict__ palm, double object_id, double rank, int64_t cand_offset, int64_t capacity,
    const int* __restrict__ counts, double* __restrict__ buf) {
  __shared__ int list[PACK_TILE];  // tile-local row → candidate offset in the tile
  const int t = threadIdx.x;
  const int b = blockIdx.x, nb = gridDim.x;
  const int W = 5 + T + D + T + 3 * T + 6;
  // survivors before this tile, and in all (fixed-order integer sums: exact)
  int64_t before = 0, total = 0;
  for (int j = t; j < nb; j += PACK_TILE) {
    const int c = counts ? counts[j] : 0;
    before += j < b ? c : 0;
    total += c;
  }
#pragma unroll
  for (int w = 1; w < 64; w <<= 1) {
    before += __shfl_xor(before, w);
    total += __shfl_xor(total, w);
  }
  const int64_t e0 = (int64_t)b * PACK_TILE;
  const bool ok = survives(e0 + t, E, T, margin);
  const unsigned long long bal = __ballot(ok);
  if (ok) list[__popcll(bal & ((1ull << t) - 1ull))] = t;
  __syncthreads();
  // field c of a record for candidate e: a branch-free address (selects, no divergent loads), so that
  // the unrolled element loop below keeps several gathers in flight per lane
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
  // rows before + [0, tile_n) of which those below `capacity` are stored
  const int tile_n = __popcll(bal);
  const int64_t n_store = before >= capacity ? 0 : (capacity - before < tile_n ? capacity - before : tile_n);
  const int n_el = (int)n_store * W;  // ≤ 64·W
  constexpr int U = 8;                // elements per lane in flight
  for (int i0 = t; i0 < n_el; i0 += U * PACK_TILE) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * PACK_TILE, n_el - 1), r = i / W;
      v[u] = field(e0 + list[r], i - r * W);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * PACK_TILE < n_el) buf[(before + 1) * W + i0 + u * PACK_TILE] = v[u];
  }
  const int64_t stored = total < capacity ? total : capacity;
  for (int64_t i = stored * W + (int64_t)b * PACK_TILE + t; i < capacity * W; i += (int64_t)nb * PACK_TILE)
    buf[W + i] = 0.0;  // unused rows
  if (b == 0)
    for (int c = t; c < W; c += PACK_TILE)
      buf[c] = c == 0 ? (double)stored : (c == 1 ? (double)total : (c == 2 ? (double)capacity : 0.0));
}

// Per-device scratch for the tile counts (grown on demand under a lock; a grown-out array is not freed,
// since a pack still queued on some stream may read it).  One scratch per device: packs on one device are
// expected one at a time in stream order (one exchange per optimise loop), not on several streams at once.
int* pack_scratch(int64_t tiles) {
  static std::mutex mu;
  static int* per_dev[64] = {};
  static int64_t cap[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (cap[dev] < tiles) {
    const int64_t want = tiles < 4096 ? 4096 : tiles;
    void* p = nullptr;
    if (hipMalloc(&p, (size_t)want * sizeof(int)) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    per_dev[dev] = static_cast<int*>(p);
    cap[dev] = want;
  }
  return per_dev[dev];
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
  const int64_t tiles = (E + PACK_TILE - 1) / PACK_TILE;
  if (tiles > INT32_MAX) return CDX_EINVAL;
  if (tiles == 0) {  // no candidates: the header and the zero rows only
    hipLaunchKernelGGL(pack_survivors_kernel, dim3(1), dim3(PACK_TILE), 0, s, (int64_t)0, (int)n_tips, (int)n_dofs,
                       margin, best_loss, q, comp, target, palm, object_id, rank, cand_offset, capacity,
                       (const int*)nullptr, buf);
    return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
  }
  int* counts = pack_scratch(tiles);
  if (!counts) return CDX_ELAUNCH;  // scratch allocation failed
  hipLaunchKernelGGL(pack_count_kernel, dim3((unsigned)tiles), dim3(PACK_TILE), 0, s, E, (int)n_tips, margin, counts);
  hipLaunchKernelGGL(pack_survivors_kernel, dim3((unsigned)tiles), dim3(PACK_TILE), 0, s, E, (int)n_tips, (int)n_dofs,
                     margin, best_loss, q, comp, target, palm, object_id, rank, cand_offset, capacity, counts, buf);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}
