/* compliancedex_amd — C ABI of the MI355X (gfx950) probabilistic-pregrasp hot path.
 *
 * Conventions:
 *   - every array argument is a DEVICE pointer owned by the caller, row-major, dense;
 *   - work is stream-ordered on the given hipStream_t (0 = null stream); nothing is
 *     allocated and nothing synchronises inside these calls;
 *   - return 0 on success, a negative CDX_E* code on a bad argument (checked before any
 *     launch), or CDX_ELAUNCH if the HIP launch itself failed.
 *
 * The reference has no FFI on this path except TorchSDF's pybind module; the entry
 * points below replace the Python/torch operators the reference calls, as cited on
 * each declaration.  Descriptor structs are plain data passed by host pointer; they
 * hold device pointers and scalars only.
 */
#ifndef CDX_H
#define CDX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* cdx_stream_t; /* == hipStream_t */

enum {
  CDX_OK = 0,
  CDX_EINVAL = -1,     /* null pointer / bad size */
  CDX_EKERNEL = -2,    /* unsupported GPIS kernel id */
  CDX_ECHAIN = -3,     /* chain too large for the fixed-capacity descriptor */
  CDX_ELAUNCH = -10    /* hipLaunch / hipGetLastError failure */
};

/* ------------------------------------------------------------------ GPIS --------
 * Replaces the GPIS object of gpis.py:4-168 (pred :43-59, compute_normal :63-87).
 * State precomputed once per object (gpis.py:33-40 fit / :162-168 load):
 *   X1     [N_pad*3]  inducing points (N_pad: multiple of CDX_NPAD_ALIGN), AoS xyz, rows >= N padded with any finite point
 *   alpha  [N_pad]    E11^{-1} y1 (zero-padded); mean = Σ alpha_j k(x, x_j) + bias
 *   Ainv   [N_pad*N_pad] E11^{-1}, symmetric, zero-padded; ∇std path
 *   Linv_t [N_pad*N_pad] (L^{-1})^T for E11 = L L^T (upper triangular), zero-padded; std path:
 *          std² = |k0 - ‖L^{-1} k‖²| (the whitened form: N² flops per query, and 1e-12 from the
 *          reference's per-call solve where k^T E11^{-1} k with an explicit inverse is 1e-7)
 *   Linv   [N_pad*N_pad] L^{-1} (lower triangular, row-major), zero-padded; closure ∇std path:
 *          E11^{-1} k = L^{-T} v from the stored whitened vector v = L^{-1} k (N² flops per query)
 * kernel: 0 = thin-plate spline 2r³-3Rr²+R³ (gpis.py:21-26, the default),
 *         1 = RBF exp(-r²/2σ²) (:16-19), 2 = 0.3·RBF + 0.7·TPS (:28-29). */
enum { CDX_KERNEL_TPS = 0, CDX_KERNEL_RBF = 1, CDX_KERNEL_JOINT = 2 };
#define CDX_NPAD_ALIGN 256   /* column width of one std-GEMM workgroup tile */

typedef struct {
  const double* X1;
  const double* alpha;
  const double* Ainv;
  const double* Linv_t;
  const double* Linv;
  int32_t N;
  int32_t N_pad;      /* multiple of CDX_NPAD_ALIGN (256), >= N */
  int32_t kernel;
  int32_t _pad;
  double R;           /* TPS radius = max pairwise training distance */
  double sigma;       /* RBF length scale */
  double bias;
  const void* screen; /* nullable: split-precision variance screen (cdx_gpis_screen_prepare) */
  double screen_delta;/* absolute bound on the screen's |Δstd²| (calibrated per state); the closure
                         screens only when screen != NULL and screen_delta > 0 */
} cdx_gpis;

/* Posterior mean and its spatial gradient at M query points (gpis.py:43-55 mean part,
 * and the autograd gradient the reference takes through it).  normal (optional) is
 * ∇mean / (‖∇mean‖ + 1e-8) — compute_normal (gpis.py:63-87), detached.
 * X [M*3]; mean [M]; grad_mean [M*3] (nullable); normal [M*3] (nullable). */
int cdx_gpis_mean(const cdx_gpis* g, const double* X, int64_t M, double* mean,
                  double* grad_mean, double* normal, cdx_stream_t stream);

/* Workspace bytes cdx_gpis_std needs for M queries. */
size_t cdx_gpis_std_workspace(const cdx_gpis* g, int64_t M);

/* Posterior standard deviation sqrt|k(0) - kᵀ E11^{-1} k| (gpis.py:56-59, the value the
 * reference returns as "var") and its gradient -sign·(E11^{-1}k)ᵀ(∂k/∂x)/std, in the whitened
 * form: v = L^{-1}k (triangular fp64 MFMA GEMM, K* generated on chip), std² = |k0 − ‖v‖²|, and
 * for the gradient E11^{-1}k = L^{-T}v (second triangular GEMM on the kept v; needs Linv, else
 * the explicit Ainv).  std [M]; grad_std [M*3] (nullable).  Workspace holds v: M·N_pad·8 bytes
 * plus partial sums (cdx_gpis_std_workspace). */
int cdx_gpis_std(const cdx_gpis* g, const double* X, int64_t M, double* std, double* grad_std,
                 void* workspace, cdx_stream_t stream);

/* On-device fit.  Replaces GPIS.fit (gpis.py:33-40):
 *   R   = max_ij ‖X1_i − X1_j‖ for the TPS / joint kernels (device scalar; 0 for RBF),
 *   E11 = K(X1, X1) + diag(noise²)   [N*N] row-major; noise [N] per point (nullable = 0).
 * N ≤ 65535. */
int cdx_gpis_fit(const double* X1, int32_t N, const double* noise, int32_t kernel, double sigma,
                 double* E11, double* R, cdx_stream_t stream);

/* Workspace bytes of cdx_gpis_factor (2·N_pad²·8). */
size_t cdx_gpis_factor_workspace(int32_t N_pad);

/* Query state from a fitted E11 (the solve gpis.py:53 repeats on every pred, done once):
 * E11 = L Lᵀ by blocked Cholesky + triangular inverse in f64, then Ainv = E11⁻¹ = L⁻ᵀL⁻¹,
 * Linv_t = L⁻ᵀ and Linv = L⁻¹ [N_pad*N_pad] zero-padded, alpha = L⁻ᵀ(L⁻¹ y1) [N_pad] zero-padded.
 * *info (device int32) = 0, or the 1-based row of the first non-positive pivot (E11 not
 * positive definite; outputs are then undefined). */
int cdx_gpis_factor(const double* E11, const double* y1, int32_t N, int32_t N_pad, void* workspace,
                    double* Ainv, double* Linv_t, double* Linv, double* alpha, int32_t* info,
                    cdx_stream_t stream);

/* Split-precision variance screen (fp16 matrix cores).  Estimates std² = k0 − ‖L⁻¹k‖² (gpis.py:56-59)
 * as k0 − ‖Ã·L⁻ᵀ + k0·colsum(L⁻ᵀ)‖² with Ã = K* − k0 generated in fp32, both operands scaled by
 * powers of two and split into two fp16 slices (three slice products, fp32 accumulation):
 * fp32-level accuracy at 32× the fp64 MFMA rate per product.  The closure uses it to skip the fp64
 * pass for fingertips that cannot be the variance cost's maximum; alone it is a throughput estimate
 * with no parity claim.  A query farther than 3.5R − max_n |x_n − centre| from the inducing points'
 * centre (TPS / joint kernels) estimates NaN.
 * cdx_gpis_screen_bytes: size of the per-state screen buffer (≈ 4·N_pad² bytes);
 * cdx_gpis_screen_prepare: fills it from g->Linv_t, g->X1, g->kernel and g->R (the descriptor's own
 *   screen field is ignored; point it at the buffer afterwards);
 * cdx_gpis_screen_var: var [M] = the estimate of k0 − ‖L⁻¹k‖² (signed), workspace
 *   cdx_gpis_screen_workspace bytes. */
size_t cdx_gpis_screen_bytes(int32_t N_pad);
int cdx_gpis_screen_prepare(const cdx_gpis* g, void* screen, cdx_stream_t stream);
/* Closure margin of a screened row at query x: screen_delta · w[b] · max(1, ‖Ṽ‖²/k0) with the distance
 * band b = ⌊4·|x − c|/ρ⌋ (last band beyond), c the inducing points' centre and ρ their largest distance
 * from it; w[CDX_SCREEN_BANDS] (host array, each in (0, 1]) is the calibrated error envelope of bands
 * ≤ b relative to the largest; cdx_gpis_screen_prepare sets them all to 1.
 * cdx_gpis_screen_info: out8 = [cx, cy, cz, SA, rq², 4/ρ, 0, 0] (host). */
#define CDX_SCREEN_BANDS 24
int cdx_gpis_screen_set_bands(const cdx_gpis* g, const double* w, cdx_stream_t stream);
int cdx_gpis_screen_info(const cdx_gpis* g, double* out8, cdx_stream_t stream);
size_t cdx_gpis_screen_workspace(const cdx_gpis* g, int64_t M);
int cdx_gpis_screen_var(const cdx_gpis* g, const double* X, int64_t M, double* var, void* workspace,
                        cdx_stream_t stream);

/* ------------------------------------------------------------------ FK ----------
 * Replaces DifferentiableRobotModel.compute_forward_kinematics(q, link_names,
 * recursive=False, offsets) (robot_model.py:224-264 with update_kinematic_state
 * :140-196, rigid_body.py:130-157, spatial_vector_algebra.py:14-136,
 * se3_so3_util.py:240-250).  Computes in float32 like the reference. */
#define CDX_MAX_BODIES 32
#define CDX_MAX_TIPS 8
#define CDX_MAX_DOFS 32

typedef struct {
  float F[9];        /* fixed rotation (Rz(yaw)·Ry(pitch))·Rx(roll), row-major */
  float t[3];        /* joint origin translation */
  float sign;        /* sign of the recognised joint axis component (0 ⇒ identity) */
  int8_t axis;       /* 0 = x, 1 = y, 2 = z */
  int8_t parent;     /* parent body index, -1 for the root */
  int8_t dof;        /* DOF index, -1 for fixed joints */
  int8_t _pad;
} cdx_body;

typedef struct {
  int32_t n_bodies;
  int32_t n_dofs;
  int32_t n_tips;
  int32_t has_offsets;
  int32_t tip_body[CDX_MAX_TIPS];
  float tip_offset[CDX_MAX_TIPS][3];
  cdx_body bodies[CDX_MAX_BODIES];
} cdx_chain;

/* q [B*n_dofs] f32 → pos [B*3*n_tips] f32, quat [B*4*n_tips] f32 (xyzw, nullable). */
int cdx_fk_forward(const cdx_chain* chain, const float* q, int64_t B, float* pos, float* quat,
                   cdx_stream_t stream);
/* Vector-Jacobian product of pos with the reference's gradient semantics (detached
 * quaternion scale, spatial_vector_algebra.py:135).  grad_pos [B*3*n_tips] → grad_q [B*n_dofs]. */
int cdx_fk_backward(const cdx_chain* chain, const float* q, int64_t B, const float* grad_pos,
                    float* grad_q, cdx_stream_t stream);

/* ------------------------------------------------------ prob-mode closure -------
 * Replaces ProbabilisticGraspOptimizer.closure (optimize_pregrasp.py:741-769) —
 * forward AND backward for E candidates — plus its callees compute_loss (:713-739),
 * force_eq_reward (:73-118), optimal_transformation_batch (:49-69),
 * compute_contact_margin (:703-710), forward_kinematics (:657-669). */
#define CDX_MAX_LEVELS 4

/* Device-resident loop counters (optional).  When cdx_problem.loop is set, every cdx_closure
 * first advances seed and step by one on the device, keys its on-device Kabsch noise by
 * (seed argument ^ loop->seed), and cdx_optimizer_step with cdx_opt_buffers.loop set takes its
 * iteration from loop->step — so a whole optimise loop can be captured once in a hipGraph and
 * replayed (fresh noise and Adam bias correction per replayed iteration). */
typedef struct {
  uint64_t seed;
  int32_t step;     /* set to -1 before the first iteration */
  int32_t _pad;
} cdx_loop;

typedef struct {
  cdx_chain chain;
  cdx_gpis gpis;
  int32_t n_levels;                     /* pregrasp levels K (3 in the reference) */
  int32_t n_query_levels;               /* distinct coefficient rows (1 if all equal) */
  int32_t level_query[CDX_MAX_LEVELS];  /* level → distinct row */
  float coeff[CDX_MAX_LEVELS][CDX_MAX_TIPS]; /* pregrasp coefficients, f32 (:644) */
  double weight[CDX_MAX_LEVELS];        /* pregrasp weights, f64 (:645) */
  float ref_q[CDX_MAX_DOFS];            /* f32 (:634) */
  float cos_mu;                         /* sqrt(1/(1+mu²)) in f32 (:111, :707) */
  int32_t gravity;                      /* dummy gravity spring on (:87-97) */
  int32_t optimize_palm;                /* palm-distance term (:760-763) */
  int32_t _pad;
  float com[3];                         /* dummy tip = COM (f32 tensor, :90-91) */
  float dummy_target_z;                 /* -M (:93) */
  float dummy_comp;                     /* gravity·mass/M (f32, :94) */
  float _pad2;
  double uncertainty;                   /* variance-cost weight (:733) */
  cdx_loop* loop;                       /* device loop counters (nullable) */
} cdx_problem;

/* Workspace bytes for E candidates. */
size_t cdx_closure_workspace(const cdx_problem* p, int64_t E);

/* One cost+grad eval for E candidates.
 * q [E*n_dofs] f64, comp [E*n_tips], target [E*n_tips*3], palm_pos [E*3], palm_ori [E*3];
 * kabsch_noise [n_levels*E*9] f64, the reference's rand_like(H) draw (:61); when NULL the
 *   noise is drawn on device from a counter-based generator keyed by (seed, row, entry).
 * Outputs: total_loss [E], total_margin [E*n_tips], pregrasp_tip [E*n_tips*3] (nullable),
 *   gradients of Σ total_loss: g_q [E*n_dofs], g_comp [E*n_tips], g_target [E*n_tips*3],
 *   g_palm_pos [E*3], g_palm_ori [E*3]; flip [n_levels*E] int32 Kabsch det<0 mask (nullable).
 * All work is ordered on `stream`; a screened call also runs the GPIS mean on a per-device side
 * stream forked from and joined back into `stream` by events (CDX_FORK_MEAN=0 disables it; 1–4
 * choose the fork point, CDX_SIDE_PRIO=-1/1 creates the side stream at the lowest / highest
 * priority — A/B switches, read once per process), so concurrent calls from several host threads
 * on one device are not supported. */
int cdx_closure(const cdx_problem* p, int64_t E, const double* q, const double* comp,
                const double* target, const double* palm_pos, const double* palm_ori,
                const double* kabsch_noise, uint64_t seed, void* workspace,
                double* total_loss, double* total_margin, double* pregrasp_tip,
                double* g_q, double* g_comp, double* g_target, double* g_palm_pos,
                double* g_palm_ori, int32_t* flip, cdx_stream_t stream);

/* Screening statistics of the last cdx_closure on this workspace (one device→host copy on the null
 * stream; prefer cdx_closure_screen_report): out[0] = all-tip rows that ran the exact fp64 whitened
 * pass, out[1] = kept rows whose split-precision estimate missed the exact value by more than its
 * margin, out[2] = all-tip rows screened; all −1 when the closure did not screen. */
int cdx_closure_screen_stats(const cdx_problem* p, int64_t E, const void* workspace, int32_t* out3);

/* The screened closure's verification record.  Every screened closure runs the exact fp64 pass for
 * each group's leader, every fingertip the selection keeps, and an AUDIT of the fingertips it discards
 * nearest the keep threshold — smallest normalised gap z = (lo − a_f)/Δ_f, lo = max_g (a_g − Δ_g), the
 * margins by which the row's estimate sits below its group's keep floor (CDX_SCREEN_AUDIT rows, default
 * 64: the lowest 1/8-octave z bins within that budget) — and checks each of those estimates against its
 * margin Δ_f.  The maximum of each group is taken over exact values.  If any check fails (a kept or
 * audited estimate off by more than Δ_f, an audited row that is its group's exact maximum, a maximum on
 * a row the exact pass did not run) the same closure REPAIRS itself: every all-tip row runs the exact
 * pass and the groups select as the unscreened closure does (repaired = 1), so no entry point returns a
 * screened result that failed a check.  A discarded row left unaudited (z ≥ min_gap) can hold its
 * group's true maximum only if its estimate is off by more than z·Δ_f; the checked rows' largest error
 * is max_ratio·Δ_f.  Fields cum_* accumulate over closures since the last cdx_closure_screen_reset (call
 * it once after allocating the workspace). */
typedef struct {
  int32_t screened;        /* 1 if the last closure on this workspace screened (else all fields 0) */
  int32_t screened_rows;   /* all-tip rows estimated by the screen */
  int32_t exact_rows;      /* rows of the exact fp64 pass: leaders + kept + audited */
  int32_t audited_rows;    /* screen-discarded rows re-checked by the exact pass */
  int32_t bound_misses;    /* kept rows whose estimate missed the exact value by more than Δ_f */
  int32_t audit_misses;    /* audited rows whose estimate missed by more than Δ_f */
  int32_t audit_flips;     /* groups whose exact maximum was an audited (screen-discarded) row */
  int32_t faults;          /* groups whose maximum fell on a row the exact pass did not run */
  double max_ratio;        /* max |estimate − exact| / Δ_f over kept rows (finite estimates) */
  double max_ratio_audit;  /* the same over audited rows */
  int64_t cum_closures;
  int64_t cum_audited_rows;
  int64_t cum_bound_misses;
  int64_t cum_audit_misses;
  int64_t cum_audit_flips;
  int64_t cum_faults;
  double cum_max_ratio;
  double cum_max_ratio_audit;
  int32_t repaired;        /* 1 if a check failed and the closure re-ran every row exactly */
  int32_t discarded_rows;  /* rows the screen discarded (audited or not) */
  double min_gap;          /* smallest z among discarded rows left unaudited (+inf: none) */
  double audit_cut;        /* every discarded row with z below this was audited */
  int64_t cum_repairs;
  int64_t cum_discarded_rows;
  double cum_min_gap;      /* smallest min_gap over the closures (+inf: none) */
} cdx_screen_report;

/* Reads the record (an async copy on `stream`, then a wait on that stream). */
int cdx_closure_screen_report(const cdx_problem* p, int64_t E, const void* workspace, cdx_screen_report* out,
                              cdx_stream_t stream);
/* Zeroes the cumulative fields and the exact pass's arrival counters (stream-ordered; REQUIRED once
 * after allocating a workspace for a screened closure); a no-op when the closure does not screen. */
int cdx_closure_screen_reset(const cdx_problem* p, int64_t E, void* workspace, cdx_stream_t stream);
/* Test hook: the next screened cdx_closure returns CDX_ELAUNCH at injection point `stage` (1: after the
 * screen / selection and the side-stream fork, 2: after the exact pass, 3: after the ∇std pass; 0 clears),
 * through the error path of a failed launch — which joins the side stream before returning. */
int cdx_debug_fail_next_closure(int32_t stage);
/* 1 if this library was built with -DCDX_AB_SWITCHES (an A/B build: it reads the CDX_* run-time switches of
 * csrc/cdx_ab.h, including CDX_SCREEN_AUDIT / CDX_SCREEN_REPAIR / CDX_NO_SCREEN), 0 for the shipped build, which
 * ignores them: every screened closure audits its discarded rows and repairs itself on a failed check. */
int cdx_ab_switches(void);

/* ------------------------------------------------------------ survivor exchange ------
 * Multi-GPU record pack (no reference counterpart — the reference is single-GPU):
 * candidates whose margins are all > 0 (the success test `opt_margin > 0`, optimize_pregrasp.py:226)
 * go to buf [(capacity + 1) * W] f64, W = 5 + n_tips + n_dofs + n_tips + 3·n_tips + 6: row 0 the header
 * [stored, survived, capacity, 0, …], rows 1.. the first `capacity` survivors in candidate order as
 * [object_id, rank, cand_offset + e, best_loss, 1, margin[T], q[D], comp[T], target[3T], palm[6]],
 * the remaining rows zero.  Two launches over 64-candidate tiles (counts, then rows), no host
 * synchronisation; the buffer feeds one all_gather.  The tile counts use a per-device scratch array: packs on
 * one device run one at a time in stream order (not concurrently on several streams). */
int cdx_pack_survivors(int64_t E, int32_t n_tips, int32_t n_dofs, const double* margin, const double* best_loss,
                       const double* q, const double* comp, const double* target, const double* palm,
                       double object_id, double rank, int64_t cand_offset, int64_t capacity, double* buf,
                       cdx_stream_t stream);

/* ------------------------------------------------------------ force_eq_reward ------
 * Replaces force_eq_reward (optimize_pregrasp.py:73-118) with optimal_transformation_batch
 * (:49-69) where the SDF / Kin / GPIS / KinGPIS optimisers (:121-513) call it directly, in f64.
 * Rows are independent: tip, target, normal [B*n_tips*3], comp [B*n_tips]; noise [B*9] is the
 * rand_like(H) draw (:61), or NULL for the on-device counter-based draw keyed by (seed, row) —
 * backward must get the same noise / seed as forward.  normal is detached (every caller passes
 * GPIS/SDF normals without a graph). */
typedef struct {
  float cos_mu;          /* sqrt(1/(1+mu²)) in f32 (:111) */
  int32_t gravity;       /* dummy gravity spring (gravity is not None, :87-97) */
  float com[3];          /* dummy tip = COM (f32 tensor, :90-91) */
  float dummy_target_z;  /* -M (:93) */
  float dummy_comp;      /* gravity·mass/M (f32, :94) */
  int32_t n_tips;
} cdx_force_eq;

/* → reward [B], margin [B*n_tips] (clamped, :112), force_norm [B*n_tips], flip [B] (nullable). */
int cdx_force_eq_forward(const cdx_force_eq* p, int64_t B, const double* tip, const double* target,
                         const double* comp, const double* normal, const double* noise, uint64_t seed,
                         double* reward, double* margin, double* force_norm, int32_t* flip,
                         cdx_stream_t stream);
/* Vector-Jacobian product: g_reward [B], g_force_norm [B*n_tips] (either nullable = 0) →
 * g_tip, g_target [B*n_tips*3], g_comp [B*n_tips] (overwritten). */
int cdx_force_eq_backward(const cdx_force_eq* p, int64_t B, const double* tip, const double* target,
                          const double* comp, const double* normal, const double* noise, uint64_t seed,
                          const double* g_reward, const double* g_force_norm, double* g_tip,
                          double* g_target, double* g_comp, cdx_stream_t stream);

/* ------------------------------------------------------------ Kin-mode iteration ------
 * KinGraspOptimizer's per-iteration cost and its backward (optimize_pregrasp.py:183-208) for E
 * candidates, one lane each, after the iteration's FK (tip = FK(q) + palm offset, float32 [E*T*3]) and
 * its three TorchSDF queries: tips vs the deflated mesh (sign1, n1), tips vs the mesh (sqdist, sign2,
 * n2, clst), targets vs the mesh (tsqdist, tsign, tclst; tsign read as [E, T]).  Returns loss [E] and
 * the force-closure margins [E*T] (f64), the blended normals [E*T*3] (nullable) and the gradients of the
 * loss w.r.t. q [E*D], target [E*T*3] and compliance [E*T] (float32, the parameters' dtype) — through
 * force_eq_reward (noise [E*9] = its rand_like draw, or NULL: drawn on device from seed), the TorchSDF
 * backward and the FK chain (float32, like the reference's autograd).  g_tip [E*T*3] (nullable) receives
 * the gradient w.r.t. the fingertips.  chain NULL: SDFGraspOptimizer's iteration (:229-320) — the tips are
 * the parameters, no ref_cost, no FK backward (q, g_q unused; g_tip required). */
typedef struct {
  cdx_force_eq fe;            /* force_eq_reward constants (mass, COM, gravity spring, friction) */
  float ref_q[CDX_MAX_DOFS];  /* ref_cost = 10·|q − ref_q| */
} cdx_kin_params;
int cdx_kin_cost(const cdx_chain* chain, const cdx_kin_params* p, int64_t E, const float* q, const float* tip,
                 const float* target, const float* comp, const int32_t* sign1, const float* n1,
                 const float* sqdist, const int32_t* sign2, const float* n2, const float* clst,
                 const float* tsqdist, const int32_t* tsign, const float* tclst, const double* noise,
                 uint64_t seed, double* loss, double* margin, float* normal, float* g_q, float* g_target,
                 float* g_comp, float* g_tip, cdx_stream_t stream);

/* ------------------------------------------------------- Kin / SDF optimiser step ------
 * One launch per iteration of KinGraspOptimizer / SDFGraspOptimizer after cdx_kin_cost (float32 like the
 * reference's parameters):
 *   1. the best-iterate update (optimize_pregrasp.py:212-222 / :299-309): per candidate, loss < opt_value
 *      (compared in double, stored as float) copies the pose, target and compliance the loss was computed on;
 *      opt_margin / opt_normal are the WHOLE batch's margin / normal of the last iteration in which ANY
 *      candidate improved (:215-217) — committed one launch late from the alternating kin_cost output slots
 *      margin[s & 1] / normal[s & 1] through the device flags any[3] (zero them before iteration 0), and by a
 *      `finalize` call after the last iteration (iteration = the iteration count; only commits);
 *   2. the optimiser step (torch's single-tensor update order in float32): rule 0 Adam (Kin, :171-176; step
 *      count iteration + 1), rule 1 RMSprop (SDF, :253-259; alpha, eps); lr 0 freezes a group;
 *   3. clamp_box: target (and, for rule 1, the tips) into [box_lb, box_ub] per fingertip (:312-314);
 *   4. rule 0 with `tips` set: the next iteration's fingertips FK(q) + palm_offset (:148), so the loop needs
 *      no separate FK launch.
 * pose is q [E*n_dofs] (rule 0) or the tips [E*n_tips*3] (rule 1); m_* are unused by RMSprop (v_* hold its
 * square averages).  chain is required for rule 0 and ignored for rule 1. */
typedef struct {
  int32_t rule;                           /* 0 Adam (Kin), 1 RMSprop (SDF) */
  int32_t clamp_box;
  double lr[3];                           /* pose, target, compliance */
  double beta1, beta2, eps;               /* Adam (eps also RMSprop's) */
  double alpha;                           /* RMSprop */
  float palm_offset[3];                   /* rule 0: tips = FK(q) + palm_offset */
  float box_lb[CDX_MAX_TIPS * 3];
  float box_ub[CDX_MAX_TIPS * 3];
  int32_t _pad;
} cdx_kin_opt;

typedef struct {                          /* device pointers, candidate-major */
  float *pose, *target, *comp;            /* parameters, in place */
  const float *g_pose, *g_target, *g_comp;
  float *m_pose, *v_pose, *m_target, *v_target, *m_comp, *v_comp;
  const double* loss;                     /* [E] this iteration's cdx_kin_cost loss */
  double* margin[2];                      /* [E*n_tips] cdx_kin_cost margin slots (iteration s wrote s & 1) */
  float* normal[2];                       /* [E*n_tips*3] cdx_kin_cost normal slots */
  float* opt_value;                       /* [E], +inf before iteration 0 */
  double* opt_margin;                     /* [E*n_tips] */
  float* opt_normal;                      /* [E*n_tips*3] */
  float *opt_pose, *opt_target, *opt_comp;
  uint32_t* any;                          /* [3] */
  float* tips;                            /* rule 0: next fingertips [E*n_tips*3] (nullable) */
  float* fk_state;                        /* rule 0, one-launch iterations with tips: the FK-walk cache, */
                                          /* cdx_kin_fk_state_bytes(E, n_tips) bytes (nullable; see below) */
} cdx_kin_opt_buffers;

/* Bytes of the FK-walk cache cdx_kin_iteration's one-launch Kin iteration uses (0: the case does not use one).  The
 * step's next-fingertip FK walk leaves each fingertip chain's joint axes / origins and final pose there, with the joint
 * angles it read, and the next iteration's FK backward takes them instead of walking the chain again when the
 * candidate's joint row still has exactly those bits and the previous iteration wrote it (else it walks): the same
 * gradient bits either way.  Any initial contents work (0xFF bytes in the Python layer); one cache per loop state and
 * chain. */
int64_t cdx_kin_fk_state_bytes(int64_t E, int32_t n_tips);

int cdx_kin_step(const cdx_chain* chain, const cdx_kin_opt* cfg, const cdx_kin_opt_buffers* buf, int64_t E,
                 int32_t n_tips, int32_t iteration, int32_t finalize, cdx_stream_t stream);
/* One whole optimiser iteration on the loop state in `buf`: cdx_kin_cost (q = pose, tip = tips for rule 0 / tip = pose
 * for rule 1; loss, margin[iteration & 1], normal[iteration & 1] and the g_* gradients into buf's buffers) followed by
 * cdx_kin_step(iteration, finalize = 0).  Two cases run as ONE launch with the same results as the two: the Kin
 * optimiser's (rule 0 = Adam, a chain, four fingertips, no clamp_box) and the SDF optimiser's (rule 1 = RMSprop, no
 * chain, four fingertips, box clamps allowed); other cases run the two launches.  chain: rule 0 only. */
int cdx_kin_iteration(const cdx_chain* chain, const cdx_kin_params* p, const cdx_kin_opt* cfg,
                      const cdx_kin_opt_buffers* buf, int64_t E, int32_t n_tips, const int32_t* sign1, const float* n1,
                      const float* sqdist, const int32_t* sign2, const float* n2, const float* clst,
                      const float* tsqdist, const int32_t* tsign, const float* tclst, const double* noise,
                      uint64_t seed, int32_t iteration, cdx_stream_t stream);

/* ------------------------------------------------------------ collision loss -------
 * Replaces ProbabilisticGraspOptimizer.compute_collision_loss (optimize_pregrasp.py:671-701):
 * anchor links by f32 FK (:674-676), palm transform R(euler XYZ)·a + palm_pos (:677-678), then
 *   Σ_pairs 1/‖a_l − a_r‖ where < pair_threshold (:679-686)
 * + Σ_anchors (1/z)·0.1 where z < floor_z (:688-691)
 * + 1/palm_z where palm_z < floor_z, if palm_term (:693-698),
 * and its gradient w.r.t. q and the palm pose.  The reference's closure leaves the call
 * commented out (:765); config 4 ("self-collision enabled") turns it on. */
#define CDX_MAX_PAIRS 28

typedef struct {
  cdx_chain chain;                      /* anchor links (collision_links + offsets) as tips */
  int32_t n_pairs;
  int32_t palm_term;                    /* optimize_palm */
  int8_t pairs[CDX_MAX_PAIRS][2];       /* anchor indices (collision_pairs) */
  double pair_threshold;                /* collision_pair_threshold (0.02) */
  double floor_z;                       /* 0.02 (:688, :694) */
} cdx_collision;

/* q [E*n_dofs] f64, palm_pos [E*3], palm_ori [E*3] → cost [E], g_q [E*n_dofs], g_palm_pos [E*3],
 * g_palm_ori [E*3] (gradients of Σ cost).  accumulate = 1 adds into the outputs (fusing the term
 * into a closure's total_loss and gradients) instead of overwriting them. */
int cdx_collision_loss(const cdx_collision* c, int64_t E, const double* q, const double* palm_pos,
                       const double* palm_ori, double* cost, double* g_q, double* g_palm_pos,
                       double* g_palm_ori, int32_t accumulate, cdx_stream_t stream);

/* ------------------------------------------------------- fused optimizer step ------
 * One launch per iteration of ProbabilisticGraspOptimizer.optimize (optimize_pregrasp.py:805-836)
 * after the closure: best-iterate update (:821-829, before the step, only when s > best_after),
 * torch.optim.Adam for the five parameter groups (:782-796; the single-tensor / foreach update
 * order: m.lerp_(g, 1-β1), v·β2 + (1-β2)·g·g, p += -lr/(1-β1^t) · m / (sqrt(v)/sqrt(1-β2^t) + eps)),
 * then the clamps compliance ≥ comp_min and target ∈ [lb, ub] (:833-834).  No host sync. */
typedef struct {
  double lr[5];                        /* q, compliance, target, palm_pos, palm_ori; 0 = frozen */
  double beta1, beta2, eps;
  double comp_min;
  double target_lb[CDX_MAX_TIPS * 3];
  double target_ub[CDX_MAX_TIPS * 3];
  int32_t clamp_target;
  int32_t best_after;                  /* best-iterate tracking from iteration best_after+1 */
} cdx_adam;

typedef struct {                       /* all device pointers, candidate-major */
  double *q, *comp, *target, *palm_pos, *palm_ori;                 /* parameters (in place) */
  const double *g_q, *g_comp, *g_target, *g_palm_pos, *g_palm_ori; /* closure gradients */
  double *m_q, *v_q, *m_comp, *v_comp, *m_target, *v_target;       /* Adam moments */
  double *m_palm_pos, *v_palm_pos, *m_palm_ori, *v_palm_ori;
  const double *total_loss, *total_margin;                         /* closure outputs */
  double *opt_value, *opt_margin, *opt_q, *opt_comp, *opt_target, *opt_palm;  /* best iterate */
  const cdx_loop* loop;                                            /* nullable: iteration from loop->step */
} cdx_opt_buffers;

/* iteration = 0-based loop index s (ignored when buf->loop is set); Adam's step count is s + 1. */
int cdx_optimizer_step(const cdx_adam* cfg, const cdx_opt_buffers* buf, int64_t E, int32_t n_dofs,
                       int32_t n_tips, int32_t iteration, cdx_stream_t stream);

/* --------------------------------------------------------------- TorchSDF -------
 * Replaces torchsdf._C.unbatched_triangle_distance_forward_cuda / _backward_cuda
 * (thirdparty/TorchSDF/torchsdf/csrc/bindings.cpp:22-27, kernels
 * unbatched_triangle_distance_cuda.cu:176-270).  float32 (the dtype the reference path uses,
 * optimize_pregrasp.py:165-168) and, through the _f64 entry points, float64 (the reference's
 * double dispatch, .cu:32-41 / :282).  Outputs are caller-allocated.
 * points [P*3], faces [F*9] → sqdist [P], sign [P] (±1), normals [P*3], clst [P*3],
 * face_idx [P] (argmin face, first minimum; nullable). */
int cdx_sdf_forward(const float* points, int64_t P, const float* faces, int64_t F,
                    float* sqdist, int32_t* sign, float* normals, float* clst,
                    int32_t* face_idx, cdx_stream_t stream);
/* grad_points = 2·grad_dist·(p − clst) (unbatched_triangle_distance_cuda.cu:256-270). */
int cdx_sdf_backward(const float* grad_dist, const float* points, const float* clst, int64_t P,
                     float* grad_points, cdx_stream_t stream);
/* float64 points / faces: the reference's double instantiation — double arithmetic except the
 * float edge parameter of point_at (.cu:171-173) and the float squared distance (.cu:237), so
 * sqdist holds float values; brute force with the reference's 512-face tile rule. */
int cdx_sdf_forward_f64(const double* points, int64_t P, const double* faces, int64_t F,
                        double* sqdist, int32_t* sign, double* normals, double* clst,
                        int32_t* face_idx, cdx_stream_t stream);
int cdx_sdf_backward_f64(const double* grad_dist, const double* points, const double* clst, int64_t P,
                         double* grad_points, cdx_stream_t stream);

/* A prepared mesh for repeated float32 queries (the SDF optimisers query the same two meshes every
 * iteration): the face records in the order of a median-split k-d tree on the face centroids (built on
 * the host: cdx_sdf_mesh_prepare copies the faces to the host and WAITS on `stream`), their disk slabs,
 * the 32-face chunks' and 512-face top nodes' bounding cylinders and balls, and the may-NaN flag of the
 * culled path.  cdx_sdf_query is cdx_sdf_forward on it — identical outputs (the face order only steers the
 * culling; ties resolve by face index).  faces must stay the ones prepared (the exact path of a NaN-capable
 * mesh scans them, and every output is recomputed from them).  mesh: cdx_sdf_mesh_bytes(F) caller-owned
 * device bytes.  cdx_sdf_query's scratch (the points' Morton sort) is `workspace` (device, at least
 * cdx_sdf_query_workspace(P) bytes — no allocation in the call), or stream-ordered scratch allocated by the
 * call when workspace is NULL. */
size_t cdx_sdf_mesh_bytes(int64_t F);
int cdx_sdf_mesh_prepare(const float* faces, int64_t F, void* mesh, cdx_stream_t stream);
size_t cdx_sdf_query_workspace(int64_t P);
/* flags of cdx_sdf_query: CDX_SDF_REUSE_ORDER — walk the points in the order the last sort on `workspace` left,
 * which must have been of P points (the same fingertips against a second mesh, or the same points a few optimiser
 * iterations earlier): the points are not sorted again.  The results do not depend on the order, only the
 * culling's speed does;
 * CDX_SDF_MESH_CULLED / CDX_SDF_MESH_EXACT — the mesh's kind as cdx_sdf_mesh_flags read it once (no NaN-capable
 * face: the culled kernel only; else the brute-force tile rule only); without either, both kernels are launched
 * and the device picks. */
/* The points' Morton order alone, into `workspace` (what cdx_sdf_query does first without CDX_SDF_REUSE_ORDER):
 * several queries of these points may then run with CDX_SDF_REUSE_ORDER concurrently on other streams, each
 * ordered after this call. */
int cdx_sdf_query_order(const float* points, int64_t P, void* workspace, size_t workspace_bytes, cdx_stream_t stream);
#define CDX_SDF_REUSE_ORDER 1
#define CDX_SDF_MESH_CULLED 2
#define CDX_SDF_MESH_EXACT 4
#define CDX_SDF_SCHED_KEEP 8 /* cdx_sdf_query_batch, first query's flags: keep the schedule's order (durations still
                                recorded; the order is recomputed on the next launch without it) */
int cdx_sdf_mesh_flags(const void* mesh, int32_t* flags, cdx_stream_t stream);  /* waits on stream */
/* Up to four cdx_sdf_query calls in one launch (the SDF / Kin optimisers' three queries per iteration): each with
 * flags CDX_SDF_REUSE_ORDER | CDX_SDF_MESH_CULLED (its workspace already holds its points' order —
 * cdx_sdf_query_order — and its mesh has no NaN-capable face); outputs identical to the separate calls. */
typedef struct cdx_sdf_batch_query {
  const void* mesh;
  const float* faces;
  int64_t F;
  const float* points;
  int64_t P;
  float* sqdist;
  int32_t* sign;
  float* normals;
  float* clst;
  int32_t* face_idx; /* nullable */
  void* workspace;
  size_t workspace_bytes;
  int32_t flags;
  int32_t _pad;
} cdx_sdf_batch_query;
/* schedule (nullable): device bytes, all zero before their first use (at least
 * cdx_sdf_batch_schedule_bytes(n, P) for the queries' point counts P[n]) that carry each point group's walk time from
 * one launch to the next — the next launch of a batch with as many groups starts the heaviest groups first (the
 * optimiser loops' same points, an iteration apart); used in stream order only, by this function only.  The outputs do
 * not depend on it. */
size_t cdx_sdf_batch_schedule_bytes(int32_t n, const int64_t* P);
int cdx_sdf_query_batch(int32_t n, const cdx_sdf_batch_query* queries, void* schedule, size_t schedule_bytes,
                        cdx_stream_t stream);
int cdx_sdf_query(const void* mesh, const float* faces, int64_t F, const float* points, int64_t P, float* sqdist,
                  int32_t* sign, float* normals, float* clst, int32_t* face_idx, void* workspace,
                  size_t workspace_bytes, int32_t flags, cdx_stream_t stream);
/* Diagnostic work counters of cdx_sdf_forward / cdx_sdf_query (float path): out3 (nullable, host) =
 * [(point, face) pairs the culled kernel evaluated exactly — each lane's greedy seed face plus the pairs
 * its slab bounds could not rule out —, pairs of brute-force scans (the exact path), points queried]; read before `enable` applies.
 * enable 1: zero the counters and count from now on (one atomic per wave); 0: stop counting; −1: only
 * read.  Against P·F per call this is the culling's work saving. */
int cdx_sdf_stats(int32_t enable, uint64_t* out3, cdx_stream_t stream);
/* Diagnostic companion of cdx_sdf_stats: chunks (32 faces) the culled kernel's waves evaluated pairs in
 * since counting was enabled, summed over waves. */
int cdx_sdf_chunk_visits(uint64_t* out, cdx_stream_t stream);

/* Library identification (gfx arch string compiled in). */
const char* cdx_version(void);

/* Per-stage kernel timing with HIP events recorded on the launch stream (off by default).
 * Stages: 0 closure query generation, 1 GPIS mean, 2 GPIS std (whitened K*·L⁻ᵀ fp64 GEMM only; in a
 * screened closure the refine pass and its merge), 3 closure cost+backward, 4 GPIS ∇std GEMM only,
 * 5 the closure's split-precision screen (fp16 GEMM + selection).  cdx_profile_read syncs on the
 * recorded events, returns the summed milliseconds and launch counts per stage (arrays of 6),
 * and clears the pool (4096 launches per stage).  `stages` is a bit mask (bit s = stage s; 0x3f
 * all, 0 off): each event record costs ≈ 5 µs of stream time, so a throughput run times only
 * the stages it reports. */
int cdx_profile_enable(int stages);
int cdx_profile_read(double* ms6, int64_t* count6);

/* sizeof(cdx_gpis), sizeof(cdx_body), sizeof(cdx_chain), sizeof(cdx_problem),
 * sizeof(cdx_collision), sizeof(cdx_adam), sizeof(cdx_opt_buffers), sizeof(cdx_force_eq),
 * sizeof(cdx_screen_report), sizeof(cdx_kin_params), sizeof(cdx_kin_opt), sizeof(cdx_kin_opt_buffers)
 * — lets a binding verify its struct layouts before the first call. */
void cdx_abi_sizes(size_t* out13);

/* Test hook: D[16×16] = A[16×4]·B[4×16] through one v_mfma_f64_16x16x4_f64 (checks the
 * fragment layout the GPIS std kernel relies on). */
int cdx_selftest_mfma_f64(const double* A, const double* B, double* D, cdx_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CDX_H */
