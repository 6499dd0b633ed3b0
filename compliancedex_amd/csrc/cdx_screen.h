// Layout of a GPIS state's screen buffer (cdx_gpis.screen, built by cdx_gpis_screen_prepare) and
// the launchers of the split-precision variance screen (cdx_screen.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "cdx.h"

namespace cdx {

constexpr int SC_BK = 16;   // K rows per stage (one v_mfma_f32_32x32x16_f16 deep)
constexpr int SC_BN = 256;  // columns per stripe (= CDX_NPAD_ALIGN)

// Column shift of the whitened products (the fp64 pass's var_shift): the N_pad − N padding
// columns, in whole 16-column blocks, sit in front of stripe 0.
__device__ __host__ inline int screen_shift(int N, int Np) { return std::min((Np - N) / 16 * 16, 256 - 16); }

__device__ __host__ inline size_t screen_align(size_t b) { return (b + 255) / 256 * 256; }

// [L: N_pad/16 × 2 slices × 2 k-halves × N_pad columns × 8 f16][csum: N_pad f64][cscale: N_pad f64]
// [X1f: N_pad float4][centre: cx, cy, cz, SA (A-operand scale), rq² (largest safe |x − centre|²),
//  4/ρ (ρ = max_n |x_n − centre|; 0 when ρ = 0), 0, 0, band weights w[CDX_SCREEN_BANDS] (below)]
inline size_t screen_bytes(int Np) {
  return screen_align((size_t)Np * Np * 4) + 2 * screen_align((size_t)Np * 8) + screen_align((size_t)Np * 16) + 256;
}

// Margin of a screened row at query x: Δ_f = screen_delta · w[b] · scale, scale = max(1, (k0 − s̃²)/k0)
// (the estimate's rounding scale ‖Ṽ‖²/k0), b = ⌊4·|x − centre|/ρ⌋ clamped to the last band (distance
// bands of a quarter object radius).  w[b] ∈ (0, 1] is the calibrated error envelope of bands ≤ b
// relative to the largest (1 everywhere until calibrated): the error grows with the distance from the
// object before ‖Ṽ‖² does, and near-object rows keep their own, smaller margin.
constexpr int SCREEN_BAND_OFF = 8;  // doubles into the centre block
__device__ __host__ inline int screen_band(const double* center, double x, double y, double z) {
  const double dx = x - center[0], dy = y - center[1], dz = z - center[2];
  const double t = sqrt(dx * dx + dy * dy + dz * dz) * center[5];
  return t < (double)(CDX_SCREEN_BANDS - 1) ? (int)t : CDX_SCREEN_BANDS - 1;  // NaN → last band
}
__device__ __host__ inline double screen_margin(double delta, const double* center, int band, double k0, double s2) {
  return delta * center[SCREEN_BAND_OFF + band] * fmax(1.0, (k0 - s2) / k0);
}

struct ScreenView {
  const void* L;
  const double* csum;
  const double* cscale;  // 1 / (SA · SB_j): the column's product scale, a power of two
  const float4* X1f;
  const double* center;
};

__device__ __host__ inline ScreenView screen_view(const cdx_gpis& g) {
  const char* p = static_cast<const char*>(g.screen);
  const size_t Np = (size_t)g.N_pad;
  const size_t oL = 0, oc = oL + screen_align(Np * Np * 4), os = oc + screen_align(Np * 8), ox = os + screen_align(Np * 8),
               oz = ox + screen_align(Np * 16);
  return ScreenView{p + oL, reinterpret_cast<const double*>(p + oc), reinterpret_cast<const double*>(p + os),
                    reinterpret_cast<const float4*>(p + ox), reinterpret_cast<const double*>(p + oz)};
}

// partials [N_pad/256][round_up(M, 256)] f64
size_t screen_ws_bytes(const cdx_gpis& g, int64_t M);
// var[m] = estimate of k0 − ‖L⁻¹k(x_m)‖² (g.screen prepared)
int screen_var_launch(const cdx_gpis& g, const double* X, int64_t M, double* var, void* ws, hipStream_t s);

// Screening statistics in the closure workspace (int32 words; "ratio" words hold the float bits of
// max |estimate − exact| / Δ_f over the rows checked, finite rows only).  Per closure (reset by the
// compaction kernel): the rows checked are every kept row and the audited rows — the discarded rows
// nearest the keep threshold (smallest normalised gap z, below).  Cumulative (reset only by
// cdx_closure_screen_reset): the same events summed over closures.
//
// Normalised gap of a discarded row f of a group: z_f = (lo − a_f)/Δ_f with lo = max_g (a_g − Δ_g), the
// margins between its estimate and the group's keep floor (> 1 for every discarded row).  The row g
// attaining lo is kept, so its exact value is known: f can hold the group's true maximum only if f's
// own estimate is off by more than z_f·Δ_f (+ (1 − ratio_g)·Δ_g).  The audit runs the rows of
// smallest z exactly; every row left out has z ≥ SS_GAP.
enum ScreenStat {
  SS_EXTRA = 0,        // rows in the exact-pass list past the G group leaders (kept + audited)
  SS_MISS = 1,         // kept rows whose finite estimate missed the exact value by more than Δ_f
  SS_AUDIT = 2,        // audited (discarded) rows
  SS_AUDIT_MISS = 3,   // audited rows whose estimate missed by more than Δ_f
  SS_AUDIT_FLIP = 4,   // groups whose exact maximum was an audited row (discarded by the screen)
  SS_FAULT = 5,        // groups whose maximum fell on a row the exact pass did not run (safe fallback)
  SS_RATIO = 6,        // max error ratio over kept rows (float bits)
  SS_RATIO_AUDIT = 7,  // max error ratio over audited rows (float bits)
  SS_REPAIR = 8,       // 1: a check above failed and the closure re-ran every all-tip row exactly
  SS_GAP = 9,          // smallest z over the discarded rows left unaudited (float bits; +inf: none)
  SS_AUDIT_CUT = 10,   // the audit's cut: every discarded row with z below it was audited (float bits)
  SS_DISCARD = 11,     // discarded rows (audited or not)
  SS_CUM = 16,         // cumulative block: [SS_CUM] closures, [SS_CUM + k] event k summed (counts),
                       // maxed (ratios) — SS_GAP as the max of 0xFFFFFFFF − bits (0: no value)
  SS_WORDS = 32
};

// Any check of this closure failed (the repair pass runs when it did).
__device__ __host__ inline bool screen_failed(const int* st) {
  return (st[SS_MISS] | st[SS_AUDIT_MISS] | st[SS_AUDIT_FLIP] | st[SS_FAULT]) != 0;
}

// The audit's row budget per closure (CDX_SCREEN_AUDIT, default 64; 0 disables the audit): the
// discarded rows are binned by z (8 bins per octave from z = 1) and the lowest bins are audited while
// their count stays ≤ the budget, plus the bin that crosses it when the total stays ≤ 4× the budget.
int screen_audit_rows();
constexpr int AUDIT_BINS = 256;
constexpr unsigned Z_NONE = 0xFFFFFFFFu;  // zkey of a kept / leader row (not an audit candidate)
__device__ __host__ inline int audit_bin(unsigned key) {
  if (key <= 0x3F800000u) return 0;  // z ≤ 1 (rounding at the keep threshold)
  const unsigned b = (key - 0x3F800000u) >> 20;
  return b < (unsigned)AUDIT_BINS ? (int)b : AUDIT_BINS - 1;
}
__device__ __host__ inline unsigned audit_bin_floor(int b) {  // float bits of the smallest z of bin b
  return b >= AUDIT_BINS ? 0x7F800000u : 0x3F800000u + ((unsigned)b << 20);
}

// Groups per workgroup of the screen's selection kernel and of its count / place (compaction) kernels: the scratch
// below and the launches in cdx_screen.hip are both sized from these.
constexpr int SCREEN_SEL_BLOCK = 64;
constexpr int SCREEN_CB_GROUPS = 256;

// Words of compaction scratch the caller allocates right behind zkey's M words (select blocks' z histograms,
// compaction block counts).
inline int64_t screen_compact_words(int64_t G) {
  return (G + SCREEN_SEL_BLOCK - 1) / SCREEN_SEL_BLOCK * AUDIT_BINS + 4 * ((G + SCREEN_CB_GROUPS - 1) / SCREEN_CB_GROUPS) + 1;
}

// Closure screening of the all-tip rows (G groups of T, M = G·T): screen partials in ws
// (screen_ws_bytes(g, M)), per-row estimate sv2, rows kept for the exact pass listed in rows[0 .. G +
// stats[SS_EXTRA]) (the G group leaders first, at position = group, then the other kept rows and the
// audited rows in group order), vpos[q] = list position or −1 (then std_[q] = the estimate), keep [G]
// masks (low byte kept, high byte audited), zkey [M + screen_compact_words(G)] the discarded rows' z (float bits;
// Z_NONE otherwise) from which the compaction picks the audited rows, then the compaction's scratch.
// after_screen(ctx), when given, runs on the host between the screen kernel's launch and the
// selection's (the closure forks its side stream there); its nonzero return is returned.
int screen_select_launch(const cdx_gpis& g, const double* X, int64_t G, int T, void* ws, double* sv2, double* std_,
                         int* vpos, int* rows, unsigned short* keep, unsigned* zkey, int* stats, hipStream_t s,
                         int (*after_screen)(void*) = nullptr, void* ctx = nullptr);
// After the refine pass (gpis_refine_launch): exact std/var of the kept and audited rows, then per
// group the ∇std row (sel = query, Xg = point, vrow = V row, always a row the exact pass ran) and the
// per-closure / cumulative statistics above.
int refine_select_launch(const cdx_gpis& g, const double* X, int64_t G, int T, const double* rpartial, int64_t M_pad,
                         const double* sv2, const int* vpos, const unsigned short* keep, double* std_, double* var,
                         int64_t* sel, double* Xg, int64_t* vrow, int* stats, hipStream_t s);

}  // namespace cdx
