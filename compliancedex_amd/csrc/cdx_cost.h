// Per-candidate prob-mode closure: cost terms, their reverse-mode gradient and the FK
// backward, in float64 (FK in float32) — one candidate per call.
//
// Reference: optimize_pregrasp.py
//   closure               :741-769    (pregrasp levels, weights, pre/palm GPIS terms)
//   compute_loss          :713-739    (seven cost terms)
//   force_eq_reward       :73-118     (dummy gravity spring, equilibrium, friction margin)
//   optimal_transformation_batch :49-69 (weighted Kabsch, SVD of H + 1e-6·noise)
//   compute_contact_margin :703-710
//   forward_kinematics    :657-669    (+ math_utils.py:68-123 euler XYZ)
// The SVD backward is torch's formula for U,V cotangents (gS = 0):
//   gH = U·[(skew(UᵀgU)∘S_k + S_j∘skew(VᵀgV)) / (S_k² − S_j²)]·Vᵀ
// evaluated on our own one-sided-Jacobi SVD (R and its gradient are invariant to the
// singular vectors' sign gauge).
#pragma once
#include "cdx_fk.h"

namespace cdx {

// ---------------------------------------------------------------- 3×3 SVD (f64)
// Compare-exchange of singular value j and j+1 (descending) with their columns of A and V, by
// selects: static register indices, where a permutation array would put A and V in scratch.
template <class Real = double>
CDX_HD void svd3_cswap(Real* s, Real* A, Real* V, int j) {
  const bool sw = s[j] < s[j + 1];
  const Real a = s[j], b = s[j + 1];
  s[j] = sw ? b : a;
  s[j + 1] = sw ? a : b;
  for (int i = 0; i < 3; ++i) {
    const Real x = A[3 * i + j], y = A[3 * i + j + 1];
    A[3 * i + j] = sw ? y : x;
    A[3 * i + j + 1] = sw ? x : y;
    const Real v = V[3 * i + j], w = V[3 * i + j + 1];
    V[3 * i + j] = sw ? w : v;
    V[3 * i + j + 1] = sw ? v : w;
  }
}

// One-sided Jacobi on the columns of A: A·V = U·diag(S), S descending.  Backward-stable
// with high relative accuracy for the small singular values the rank-1-plus-noise
// Kabsch matrices of the reference's initial configuration have.  Real = double (the prob-mode closure: the
// reference's float64 tensors) or float (the Kin / SDF optimisers: the reference's float32 tensors), with the
// rotation-skip and convergence thresholds at the type's epsilon.
template <class Real>
struct Svd3Tol;
template <>
struct Svd3Tol<double> {
  static constexpr double skip = 1e-17, stop = 1e-16;
};
template <>
struct Svd3Tol<float> {
  static constexpr float skip = 1e-8f, stop = 6e-8f;
};
CDX_HD double svd3_rsqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return rsqrt(x);
#else
  return 1.0 / sqrt(x);
#endif
}
CDX_HD float svd3_rsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return rsqrtf(x);
#else
  return 1.0f / sqrtf(x);
#endif
}
template <class Real = double>
CDX_HD void svd3(const Real* H, Real* U, Real* S, Real* V) {
#if defined(CDX_DIAG_NOSVD)  // timing-only diagnostic build (outputs wrong): the level kernel without its SVD
  for (int i = 0; i < 9; ++i) { U[i] = V[i] = (i % 4 == 0) ? Real(1) : Real(0); }
  S[0] = Real(3) + H[0]; S[1] = Real(2) + H[4]; S[2] = Real(1) + H[8];
  return;
#endif
  Real A[9];
  for (int i = 0; i < 9; ++i) { A[i] = H[i]; V[i] = (i % 4 == 0) ? Real(1) : Real(0); }
  for (int sweep = 0; sweep < 12; ++sweep) {
#if defined(CDX_SVD_JACOBI_R5)  // (A/B: the round-5 rotation — 3 roots and 4 divisions per pair)
    Real off = Real(0);
#else
    bool more = false;
#endif
    for (int pr = 0; pr < 3; ++pr) {
      const int p = pr == 2 ? 1 : 0, qq = pr == 0 ? 1 : 2;
      Real a = 0, b = 0, g = 0;
      for (int i = 0; i < 3; ++i) {
        a += A[3 * i + p] * A[3 * i + p];
        b += A[3 * i + qq] * A[3 * i + qq];
        g += A[3 * i + p] * A[3 * i + qq];
      }
      if (g == Real(0)) continue;
#if defined(CDX_SVD_JACOBI_R5)
      const Real rel = fabs(g) / sqrt(a * b);
      off = rel > off ? rel : off;
      if (rel < Svd3Tol<Real>::skip) continue;
      const Real zeta = (b - a) / (Real(2) * g);
      const Real t = (zeta >= 0 ? Real(1) : Real(-1)) / (fabs(zeta) + sqrt(Real(1) + zeta * zeta));
      const Real c = Real(1) / sqrt(Real(1) + t * t), s = c * t;
#else
      // the same rotation with one root, one division and one reciprocal root: |g|/sqrt(ab) compared squared,
      // t = sgn(ζ)/(|ζ| + sqrt(1 + ζ²)) with ζ = (b − a)/2g written as sgn(ζ)·2|g| / (|b − a| + sqrt((b − a)² + 4g²)),
      // c = rsqrt(1 + t²) — the Jacobi SVD's divisions and roots were ≈ 17 µs of the Kin cost kernel (r05bd)
      const Real g2 = g * g, ab = a * b;
      if (!(g2 < Svd3Tol<Real>::stop * Svd3Tol<Real>::stop * ab)) more = true;
      if (g2 < Svd3Tol<Real>::skip * Svd3Tol<Real>::skip * ab) continue;
      const Real d = b - a, ag = fabs(g);
      const Real zs = (d >= 0) == (g >= 0) || d == Real(0) ? Real(2) * ag : Real(-2) * ag;  // sgn(ζ)·2|g|
      const Real t = zs / (fabs(d) + sqrt(d * d + Real(4) * g2));
      const Real c = svd3_rsqrt(Real(1) + t * t), s = c * t;
#endif
      for (int i = 0; i < 3; ++i) {
        const Real ap = A[3 * i + p], aq = A[3 * i + qq];
        A[3 * i + p] = c * ap - s * aq;
        A[3 * i + qq] = s * ap + c * aq;
        const Real vp = V[3 * i + p], vq = V[3 * i + qq];
        V[3 * i + p] = c * vp - s * vq;
        V[3 * i + qq] = s * vp + c * vq;
      }
    }
#if defined(CDX_SVD_JACOBI_R5)
    if (off < Svd3Tol<Real>::stop) break;
#else
    if (!more) break;
#endif
  }
  Real s[3];
  for (int j = 0; j < 3; ++j) s[j] = sqrt(A[j] * A[j] + A[3 + j] * A[3 + j] + A[6 + j] * A[6 + j]);
  // descending bubble network (0,1), (1,2), (0,1) with strict comparisons: the permutation of a
  // bubble sort of the column indices by s
  svd3_cswap(s, A, V, 0);
  svd3_cswap(s, A, V, 1);
  svd3_cswap(s, A, V, 0);
  for (int j = 0; j < 3; ++j) {
    S[j] = s[j];
    for (int i = 0; i < 3; ++i) U[3 * i + j] = s[j] > 0 ? A[3 * i + j] / s[j] : Real(0);
  }
  if (!(S[2] > 0)) {  // exactly singular: complete U with the cross product
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
  }
}

template <class Real = double>
CDX_HD Real det3(const Real* m) {
  return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// Kabsch state kept for the backward pass.
template <class Real = double>
struct KabschTapeT {
  Real U[9], S[3], V[9];
  Real d;  // +1, or -1 when det(V·Uᵀ) < 0 (the reference's `mask`, :64-66)
};
using KabschTape = KabschTapeT<double>;

// R = V·diag(1,1,d)·Uᵀ of H' = H + 1e-6·noise (the noise draw in Real, as the reference's rand_like(H)).
template <class Real = double>
CDX_HD void kabsch_rotation(const Real* H, const double* noise, KabschTapeT<Real>& tp, Real* R) {
  Real Hn[9];
  for (int i = 0; i < 9; ++i) Hn[i] = H[i] + Real(1e-6) * (Real)noise[i];
  svd3(Hn, tp.U, tp.S, tp.V);
  Real R0[9];
  mat3_mul_nt(tp.V, tp.U, R0);
  tp.d = det3(R0) < Real(0) ? Real(-1) : Real(1);
  Real Vd[9];
  for (int i = 0; i < 3; ++i) { Vd[3 * i] = tp.V[3 * i]; Vd[3 * i + 1] = tp.V[3 * i + 1]; Vd[3 * i + 2] = tp.V[3 * i + 2] * tp.d; }
  mat3_mul_nt(Vd, tp.U, R);
}

// gH from gR through R = V·D·Uᵀ and the SVD.
template <class Real = double>
CDX_HD void kabsch_rotation_bwd(const KabschTapeT<Real>& tp, const Real* gR, Real* gH) {
  const Real* U = tp.U;
  const Real* V = tp.V;
  const Real* S = tp.S;
  // gU = gRᵀ·V·D ; gV = gR·U·D
  Real gU[9], gV[9], t[9];
  mat3_mul_tn(gR, V, t);
  for (int i = 0; i < 3; ++i) { gU[3 * i] = t[3 * i]; gU[3 * i + 1] = t[3 * i + 1]; gU[3 * i + 2] = t[3 * i + 2] * tp.d; }
  mat3_mul(gR, U, t);
  for (int i = 0; i < 3; ++i) { gV[3 * i] = t[3 * i]; gV[3 * i + 1] = t[3 * i + 1]; gV[3 * i + 2] = t[3 * i + 2] * tp.d; }
  Real UgU[9], VgV[9];
  mat3_mul_tn(U, gU, UgU);
  mat3_mul_tn(V, gV, VgV);
  Real X[9];
  for (int j = 0; j < 3; ++j)
    for (int k = 0; k < 3; ++k) {
      if (j == k) { X[3 * j + k] = Real(0); continue; }
      const Real sku = UgU[3 * j + k] - UgU[3 * k + j];
      const Real skv = VgV[3 * j + k] - VgV[3 * k + j];
      X[3 * j + k] = (sku * S[k] + S[j] * skv) / (S[k] * S[k] - S[j] * S[j]);
    }
  Real UX[9];
  mat3_mul(U, X, UX);
  mat3_mul_nt(UX, V, gH);
}

// ------------------------------------------------------------- euler XYZ (f64)
CDX_HD void rot_axis_d(int axis, double a, double* R, double* dR) {
  const double c = cos(a), s = sin(a);
  for (int i = 0; i < 9; ++i) { R[i] = 0.0; dR[i] = 0.0; }
  if (axis == 0) {
    R[0] = 1; R[4] = c; R[5] = -s; R[7] = s; R[8] = c;
    dR[4] = -s; dR[5] = -c; dR[7] = c; dR[8] = -s;
  } else if (axis == 1) {
    R[0] = c; R[2] = s; R[4] = 1; R[6] = -s; R[8] = c;
    dR[0] = -s; dR[2] = c; dR[6] = -c; dR[8] = -s;
  } else {
    R[0] = c; R[1] = -s; R[3] = s; R[4] = c; R[8] = 1;
    dR[0] = -s; dR[1] = -c; dR[3] = c; dR[4] = -s;
  }
}

// R = (Rx(a)·Ry(b))·Rz(c)  (math_utils.py:97-123); optionally the three partials.
CDX_HD void euler_xyz(const double* ang, double* R, double* dRa, double* dRb, double* dRc) {
  double X[9], dX[9], Y[9], dY[9], Z[9], dZ[9], XY[9];
  rot_axis_d(0, ang[0], X, dX);
  rot_axis_d(1, ang[1], Y, dY);
  rot_axis_d(2, ang[2], Z, dZ);
  mat3_mul(X, Y, XY);
  mat3_mul(XY, Z, R);
  if (dRa) {
    double t[9];
    mat3_mul(dX, Y, t); mat3_mul(t, Z, dRa);
    mat3_mul(X, dY, t); mat3_mul(t, Z, dRb);
    mat3_mul(XY, dZ, dRc);
  }
}

// --------------------------------------------------------------- GPIS at a point
struct GpisPoint {
  double mean, gmean[3];
  double std, gstd[3];   // only for all-tip queries
  double normal[3];
};

// ------------------------------------------------------------ closure per candidate
// Query-array layout (T tips, Lq distinct coefficient rows, E candidates):
//   all-tip row u : u·E·T + e·T + f        target : Lq·E·T + e·T + f
//   pregrasp      : (Lq+1)·E·T + e·T + f    palm   : (Lq+2)·E·T + e
CDX_HD int64_t q_alltip(int u, int64_t e, int f, int64_t E, int T) { return (int64_t)u * E * T + e * T + f; }
CDX_HD int64_t q_target(int Lq, int64_t e, int f, int64_t E, int T) { return (int64_t)Lq * E * T + e * T + f; }
CDX_HD int64_t q_pre(int Lq, int64_t e, int f, int64_t E, int T) { return (int64_t)(Lq + 1) * E * T + e * T + f; }
CDX_HD int64_t q_palm(int Lq, int64_t e, int64_t E, int T) { return (int64_t)(Lq + 2) * E * T + e; }
CDX_HD int64_t n_queries(const cdx_problem& P, int64_t E) {
  const int T = P.chain.n_tips;
  return (int64_t)(P.n_query_levels + 2) * E * T + (P.optimize_palm ? E : 0);
}

// Pregrasp fingertips in world frame for candidate e: f32 FK, cast to f64, palm transform.
CDX_HD void pregrasp_tips(const cdx_problem& P, const double* q, const double* palm_pos, const double* palm_ori,
                          double (*tip)[3], float (*tl)[3], double* Rp) {
  const int T = P.chain.n_tips;
  float qf[CDX_MAX_DOFS];
  for (int i = 0; i < P.chain.n_dofs; ++i) qf[i] = (float)q[i];
  euler_xyz(palm_ori, Rp, nullptr, nullptr, nullptr);
  for (int f = 0; f < T; ++f) {
    fk_tip(P.chain, f, qf, tl[f], nullptr);
    const double v[3] = {(double)tl[f][0], (double)tl[f][1], (double)tl[f][2]};
    double w[3];
    mat3_vec(Rp, v, w);
    for (int i = 0; i < 3; ++i) tip[f][i] = w[i] + palm_pos[i];
  }
}

// ‖q − ref_q‖ with ref_q float32 (:732); dq receives q − ref_q.
CDX_HD double ref_dist(const cdx_problem& P, const double* q, double* dq) {
  double qn2 = 0.0;
  for (int i = 0; i < P.chain.n_dofs; ++i) {
    dq[i] = q[i] - (double)P.ref_q[i];
    qn2 += dq[i] * dq[i];
  }
  return sqrt(qn2);
}

struct CandidateIn {
  const double *q, *comp, *target, *palm_pos, *palm_ori;  // this candidate's rows
  const double* noise;                                     // [K][9] for this candidate (stride via noise_stride)
  int64_t noise_stride;                                    // doubles between levels
  const double* rot = nullptr;  // this level's Kabsch record (ForceEq::save_rotation), or null: SVD inline
};

struct CandidateOut {
  double loss;
  double margin[CDX_MAX_TIPS];
  double g_q[CDX_MAX_DOFS];
  double g_comp[CDX_MAX_TIPS];
  double g_target[CDX_MAX_TIPS][3];
  double g_palm_pos[3];
  double g_palm_ori[3];
  int flip[CDX_MAX_LEVELS];
};

// ------------------------------------------------------------ force_eq_reward
// force_eq_reward (:73-118) with optimal_transformation_batch (:49-69) for one row: the weighted
// Kabsch fit of [tips, dummy] onto [targets, dummy] (dummy gravity spring: tip = COM, target z = −M,
// weight gravity·mass/M, all float32 tensors in the reference), equilibrium tips, friction-cone
// margin clamp(ang − cos_mu, −0.9999) and reward Σ 0.2·log(ang+1) + 0.8·log(margin+1).  forward()
// keeps the tape; backward() takes dL/dreward and dL/dforce_norm and ACCUMULATES into the tip,
// target and compliance gradients (normals are detached, as every caller passes them).
struct ForceEqParams {
  double cos_mu;
  int gravity;
  double com[3];
  double dummy_target_z;
  double dummy_comp;
};

CDX_HD ForceEqParams force_eq_params(const cdx_problem& P) {
  ForceEqParams fp;
  fp.cos_mu = (double)P.cos_mu;
  fp.gravity = P.gravity;
  for (int i = 0; i < 3; ++i) fp.com[i] = (double)P.com[i];
  fp.dummy_target_z = (double)P.dummy_target_z;
  fp.dummy_comp = (double)P.dummy_comp;
  return fp;
}

// NT: fingertip count at compile time (0: runtime, up to CDX_MAX_TIPS); G: gravity spring at
// compile time (0 / 1; -1: runtime) — with both fixed every loop has a constant trip count.
template <int NT, int G = -1, class Real = double>
struct ForceEq {
  static constexpr int NTA = NT > 0 ? NT : CDX_MAX_TIPS;
  int T_rt, NP_rt;
  // The tape keeps what backward cannot cheaply recompute; the weighted centred points, R·S1,
  // the residuals, directions, rotated normals and forces are recomputed there by the same
  // expressions (bit-identical values) — keeping them made the level kernel spill to scratch.
  Real S1[NTA + 1][3], S2[NTA + 1][3], w[NTA + 1], n[NTA][3];
  Real c1[3], c2[3];
  KabschTapeT<Real> tp;
  Real R[9], W, t[3];
  Real dn[NTA], ang[NTA], mpre[NTA], margin[NTA], fn[NTA];
  Real reward;
  int flip;

  // The points, weights and centroids of the weighted Kabsch fit (everything before the SVD).
  CDX_HDM void setup(const ForceEqParams& fp, int T_, const Real (*tip)[3], const Real* target, const Real* comp,
                     const Real (*nrm)[3]) {
    T_rt = T_;
    const int T = NT > 0 ? NT : T_;
    const bool grav = G >= 0 ? G != 0 : fp.gravity != 0;
    NP_rt = grav ? T + 1 : T;
    const int NP = (NT > 0 && G >= 0) ? (G ? NT + 1 : NT) : NP_rt;
#pragma unroll
    for (int f = 0; f < T; ++f) {
      for (int i = 0; i < 3; ++i) { S1[f][i] = tip[f][i]; S2[f][i] = target[3 * f + i]; n[f][i] = nrm ? nrm[f][i] : Real(0); }
      w[f] = comp[f];
    }
    if (grav) {
      for (int i = 0; i < 3; ++i) S1[T][i] = (Real)fp.com[i];
      S2[T][0] = 0.0; S2[T][1] = 0.0; S2[T][2] = (Real)fp.dummy_target_z;
      w[T] = (Real)fp.dummy_comp;
    }
    c1[0] = c1[1] = c1[2] = 0.0;
    c2[0] = c2[1] = c2[2] = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i)
      for (int j = 0; j < 3; ++j) { c1[j] += S1[i][j]; c2[j] += S2[i][j]; }
    for (int j = 0; j < 3; ++j) { c1[j] /= NP; c2[j] /= NP; }
  }

  // H = Σ w_i (S1_i − c1)(w_i (S2_i − c2))ᵀ, then the rotation and its tape (R = V·D·Uᵀ of H + 1e-6·noise).
  CDX_HDM void rotation(const double* noise) {
    const int NP = (NT > 0 && G >= 0) ? (G ? NT + 1 : NT) : NP_rt;
    Real H[9];
    {
      Real Pm[NTA + 1][3], Qm[NTA + 1][3];
#pragma unroll
      for (int i = 0; i < NP; ++i)
        for (int j = 0; j < 3; ++j) { Pm[i][j] = w[i] * (S1[i][j] - c1[j]); Qm[i][j] = w[i] * (S2[i][j] - c2[j]); }
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          Real acc = 0.0;
#pragma unroll
          for (int i = 0; i < NP; ++i) acc += Pm[i][r] * Qm[i][c];
          H[3 * r + c] = acc;
        }
    }
    {
      // svd3 sorts with data-dependent indices: run it on a separate tape so that only this small
      // object, not the whole ForceEq, has to live in scratch
      KabschTapeT<Real> t_;
      kabsch_rotation(H, noise, t_, R);
      tp = t_;
    }
  }

  // The rotation stage as a record of KABSCH_RECORD doubles [U, S, V, d, R] (closure_kabsch_kernel
  // computes it ahead of the level kernel) and back.
  static constexpr int KABSCH_RECORD = 32;
  CDX_HDM void save_rotation(double* rec) const {
    for (int i = 0; i < 9; ++i) { rec[i] = tp.U[i]; rec[12 + i] = tp.V[i]; rec[22 + i] = R[i]; }
    for (int i = 0; i < 3; ++i) rec[9 + i] = tp.S[i];
    rec[21] = tp.d;
  }
  CDX_HDM void load_rotation(const double* rec) {
    for (int i = 0; i < 9; ++i) { tp.U[i] = (Real)rec[i]; tp.V[i] = (Real)rec[12 + i]; R[i] = (Real)rec[22 + i]; }
    for (int i = 0; i < 3; ++i) tp.S[i] = (Real)rec[9 + i];
    tp.d = (Real)rec[21];
  }

  // Everything after the rotation: translation, equilibrium residuals, friction margins, reward.
  CDX_HDM void finish(const ForceEqParams& fp, const Real* comp) {
    const int T = NT > 0 ? NT : T_rt;
    const int NP = (NT > 0 && G >= 0) ? (G ? NT + 1 : NT) : NP_rt;
    flip = tp.d < Real(0) ? 1 : 0;
    W = 0.0;
    Real num[3] = {0, 0, 0};
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      W += w[i];
      Real rs[3];
      mat3_vec(R, S1[i], rs);
      for (int j = 0; j < 3; ++j) num[j] += w[i] * (S2[i][j] - rs[j]);
    }
    for (int j = 0; j < 3; ++j) t[j] = num[j] / W;
    reward = 0.0;
#pragma unroll
    for (int f = 0; f < T; ++f) {
      Real diff[3], dir[3], ne[3], force[3];
      residual(f, diff);
      dn[f] = sqrt(dot3(diff, diff));
      for (int i = 0; i < 3; ++i) { dir[i] = diff[i] / dn[f]; force[i] = comp[f] * (-diff[i]); }
      mat3_vec(R, n[f], ne);
      ang[f] = dot3(dir, ne);
      mpre[f] = ang[f] - (Real)fp.cos_mu;
      margin[f] = mpre[f] < Real(-0.9999) ? Real(-0.9999) : mpre[f];
      fn[f] = sqrt(dot3(force, force));
      reward += Real(0.2) * log(ang[f] + Real(1)) + Real(0.8) * log(margin[f] + Real(1));
    }
  }

  // rot: a record save_rotation wrote for the same inputs, or null (the SVD runs here).
  CDX_HDM void forward(const ForceEqParams& fp, int T_, const Real (*tip)[3], const Real* target,
                      const Real* comp, const Real (*nrm)[3], const double* noise, const double* rot = nullptr) {
    setup(fp, T_, tip, target, comp, nrm);
    if (rot)
      load_rotation(rot);
    else
      rotation(noise);
    finish(fp, comp);
  }

  // diff_f = R·S1_f + t − target_f (S2_f holds target_f)
  CDX_HDM void residual(int f, Real* diff) const {
    Real rs[3];
    mat3_vec(R, S1[f], rs);
    for (int i = 0; i < 3; ++i) diff[i] = rs[i] + t[i] - S2[f][i];
  }

  CDX_HDM void backward(Real g_rw, const Real* g_fn, const Real* comp, Real (*g_tip)[3], Real (*g_target)[3],
                       Real* g_comp) const {
    const int T = NT > 0 ? NT : T_rt;
    const int NP = (NT > 0 && G >= 0) ? (G ? NT + 1 : NT) : NP_rt;
    Real gR[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g_t[3] = {0, 0, 0};
    Real g_S1[NTA + 1][3], g_S2[NTA + 1][3], g_w[NTA + 1];
#pragma unroll
    for (int i = 0; i < NP; ++i) { g_S1[i][0] = g_S1[i][1] = g_S1[i][2] = 0; g_S2[i][0] = g_S2[i][1] = g_S2[i][2] = 0; g_w[i] = 0; }
#pragma unroll
    for (int f = 0; f < T; ++f) {
      Real diff[3], dir[3], ne[3];
      residual(f, diff);
      for (int i = 0; i < 3; ++i) dir[i] = diff[i] / dn[f];
      mat3_vec(R, n[f], ne);
      Real gang = g_rw * Real(0.2) / (ang[f] + Real(1));
      if (mpre[f] >= Real(-0.9999)) gang += g_rw * Real(0.8) / (margin[f] + Real(1));
      Real gdiff[3] = {0, 0, 0};
      // force norm → force = −comp·diff
      if (fn[f] > 0) {
        Real gforce[3];
        for (int i = 0; i < 3; ++i) gforce[i] = g_fn[f] * (comp[f] * (-diff[i])) / fn[f];
        g_w[f] += -dot3(gforce, diff);
        for (int i = 0; i < 3; ++i) gdiff[i] += -comp[f] * gforce[i];
      }
      // ang = dir·ne ; ne = R·n (n detached)
      Real gdir[3], gne[3];
      for (int i = 0; i < 3; ++i) { gdir[i] = gang * ne[i]; gne[i] = gang * dir[i]; }
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) gR[3 * r + c] += gne[r] * n[f][c];
      const Real pd = dot3(dir, gdir);
      for (int i = 0; i < 3; ++i) gdiff[i] += (gdir[i] - dir[i] * pd) / dn[f];
      // diff = R·S1_f + t − target_f
      for (int i = 0; i < 3; ++i) { g_t[i] += gdiff[i]; g_target[f][i] -= gdiff[i]; }
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) gR[3 * r + c] += gdiff[r] * S1[f][c];
      Real rt[3];
      mat3t_vec(R, gdiff, rt);
      for (int i = 0; i < 3; ++i) g_S1[f][i] += rt[i];
    }
    // t = Σ w_i (S2_i − R·S1_i) / W
    {
      Real gnum[3] = {g_t[0] / W, g_t[1] / W, g_t[2] / W};
      const Real gW = -dot3(g_t, t) / W;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        Real rs[3];
        mat3_vec(R, S1[i], rs);
        Real r_i[3] = {S2[i][0] - rs[0], S2[i][1] - rs[1], S2[i][2] - rs[2]};
        g_w[i] += gW + dot3(gnum, r_i);
        for (int j = 0; j < 3; ++j) g_S2[i][j] += w[i] * gnum[j];
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c) gR[3 * r + c] -= w[i] * gnum[r] * S1[i][c];
        Real rt[3], wg[3] = {w[i] * gnum[0], w[i] * gnum[1], w[i] * gnum[2]};
        mat3t_vec(R, wg, rt);
        for (int j = 0; j < 3; ++j) g_S1[i][j] -= rt[j];
      }
    }
    // R ← SVD(H') ← H = Σ P_i Q_iᵀ
    Real gH[9];
    kabsch_rotation_bwd(tp, gR, gH);
    Real g_c1[3] = {0, 0, 0}, g_c2[3] = {0, 0, 0};
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      Real gP[3], gQ[3];
      Real d1[3] = {S1[i][0] - c1[0], S1[i][1] - c1[1], S1[i][2] - c1[2]};
      Real d2[3] = {S2[i][0] - c2[0], S2[i][1] - c2[1], S2[i][2] - c2[2]};
      const Real Pm[3] = {w[i] * d1[0], w[i] * d1[1], w[i] * d1[2]}, Qm[3] = {w[i] * d2[0], w[i] * d2[1], w[i] * d2[2]};
      mat3_vec(gH, Qm, gP);
      mat3t_vec(gH, Pm, gQ);
      g_w[i] += dot3(gP, d1) + dot3(gQ, d2);
      for (int j = 0; j < 3; ++j) {
        g_S1[i][j] += w[i] * gP[j];
        g_c1[j] -= w[i] * gP[j];
        g_S2[i][j] += w[i] * gQ[j];
        g_c2[j] -= w[i] * gQ[j];
      }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i)
      for (int j = 0; j < 3; ++j) { g_S1[i][j] += g_c1[j] / NP; g_S2[i][j] += g_c2[j] / NP; }
#pragma unroll
    for (int f = 0; f < T; ++f) {
      for (int i = 0; i < 3; ++i) { g_tip[f][i] += g_S1[f][i]; g_target[f][i] += g_S2[f][i]; }
      g_comp[f] += g_w[f];
    }
  }
};

// One pregrasp level of compute_loss (:713-739) for one candidate, forward AND backward with
// dL/dl_k = w_k: returns l_k, margin_k, the Kabsch mask and the level's gradient w.r.t. the
// pregrasp tips, targets and compliances.  NT = fingertip count at compile time (0: runtime).
struct LevelOut {
  double l;
  double margin[CDX_MAX_TIPS];
  double g_tip[CDX_MAX_TIPS][3];
  double g_target[CDX_MAX_TIPS][3];
  double g_comp[CDX_MAX_TIPS];
  int flip;
};

// VAR = false leaves the variance cost out of l and of the gradients (its loss term is the last operand of
// l's left-to-right sum, so adding uncertainty·lmax to the record later gives l bit for bit): the closure's
// combine kernel adds it once ∇std is known, so this level kernel needs neither std nor ∇std and can run
// beside the std passes (cdx_closure.hip, var_late()).
template <int NT, typename GpisAt, int G = -1, bool PRE = false, bool VAR = true>
CDX_HD void level_fwd_bwd(const cdx_problem& P, int k, const CandidateIn& in, const double (*tip)[3], double qnorm,
                          GpisAt gp, LevelOut& o) {
  constexpr int NTA = NT > 0 ? NT : CDX_MAX_TIPS;
  const int T = NT > 0 ? NT : P.chain.n_tips;
  const double cos_mu = (double)P.cos_mu;
  for (int f = 0; f < T; ++f) {
    for (int i = 0; i < 3; ++i) { o.g_target[f][i] = 0.0; o.g_tip[f][i] = 0.0; }
    o.g_comp[f] = 0.0;
  }
  const int u = P.level_query[k];
  const double wk = P.weight[k];
  // ---- forward of compute_loss for this level
  double a[NTA][3], d[NTA], s[NTA], n[NTA][3], td[NTA];
  for (int f = 0; f < T; ++f) {
    const double c = (double)P.coeff[k][f];
    for (int i = 0; i < 3; ++i) a[f][i] = in.target[3 * f + i] + c * (tip[f][i] - in.target[3 * f + i]);
    const GpisPoint& ga = gp(0, u, f);
    d[f] = ga.mean;
    s[f] = ga.std;
    for (int i = 0; i < 3; ++i) n[f][i] = ga.normal[i];
    td[f] = gp(1, 0, f).mean;
  }
  ForceEq<NT, G> fe;
  if constexpr (PRE) {  // the Kabsch record is given (in.rot): no SVD code in this instantiation
    fe.setup(force_eq_params(P), T, a, in.target, in.comp, n);
    fe.load_rotation(in.rot);
    fe.finish(force_eq_params(P), in.comp);
  } else {
    fe.forward(force_eq_params(P), T, a, in.target, in.comp, n, in.noise + k * in.noise_stride, in.rot);
  }
  o.flip = fe.flip;
  // contact margin (unclamped), from the copies ForceEq keeps (fe.S1 = a, fe.S2 = target, fe.n = n):
  // the backward recomputes it the same way, so a and n need not stay live through the SVD
  auto contact = [&](int f, double* cdir, double& cdn, double& cang) {
    double cd[3];
    for (int i = 0; i < 3; ++i) cd[i] = fe.S1[f][i] - fe.S2[f][i];
    cdn = sqrt(dot3(cd, cd));
    for (int i = 0; i < 3; ++i) cdir[i] = cd[i] / cdn;
    cang = dot3(cdir, fe.n[f]);
  };
  double creward = 0.0;
  for (int f = 0; f < T; ++f) {
    double cdir[3], cdn, cang;
    contact(f, cdir, cdn, cang);
    creward += 0.1 * log(cang + 1) + 0.9 * log(cang - cos_mu + 1);
  }
  // force cost: −Σ clamp(fn·softmin(fn), max=10)
  const double* fn = fe.fn;
  double zmax = -fn[0];
  for (int f = 1; f < T; ++f) zmax = -fn[f] > zmax ? -fn[f] : zmax;
  double ez[NTA], esum = 0.0;
  for (int f = 0; f < T; ++f) { ez[f] = exp(-fn[f] - zmax); esum += ez[f]; }
  double sm[NTA], v[NTA], fcost = 0.0;
  for (int f = 0; f < T; ++f) {
    sm[f] = ez[f] / esum;
    v[f] = fn[f] * sm[f];
    fcost += v[f] > 10.0 ? 10.0 : v[f];
  }
  fcost = -fcost;
  // variance cost: uncertainty · max_f log(100 std)
  int fmax = 0;
  double lmax = 0.0;
  if constexpr (VAR) {
    lmax = log(100 * s[0]);
    for (int f = 1; f < T; ++f) {
      const double lv = log(100 * s[f]);
      if (lv > lmax) { lmax = lv; fmax = f; }
    }
  }
  double dcost = 0.0, tcost = 0.0;
  for (int f = 0; f < T; ++f) { dcost += fabs(d[f]); tcost += td[f]; }
  const double l0 = -fe.reward * 200.0 + 1000 * dcost + 20 * tcost + (-creward * 200.0) + fcost + qnorm * 10.0;
  o.l = VAR ? l0 + P.uncertainty * lmax : l0;
  for (int f = 0; f < T; ++f) o.margin[f] = fe.margin[f];

  // ---- backward of this level with dL/dl = wk
  double g_a[NTA][3];
  for (int f = 0; f < T; ++f) g_a[f][0] = g_a[f][1] = g_a[f][2] = 0.0;
  // dist / tar_dist / variance (GPIS gradients at the query points)
  for (int f = 0; f < T; ++f) {
    const GpisPoint& ga = gp(0, u, f);
    const double sg = d[f] > 0 ? 1.0 : (d[f] < 0 ? -1.0 : 0.0);
    const double gd = wk * 1000.0 * sg;
    for (int i = 0; i < 3; ++i) g_a[f][i] += gd * ga.gmean[i];
    const GpisPoint& gt = gp(1, 0, f);
    for (int i = 0; i < 3; ++i) o.g_target[f][i] += wk * 20.0 * gt.gmean[i];
  }
  if constexpr (VAR) {
    // (fmax is data-dependent: the update is selected per fingertip so g_a keeps static indices)
    const GpisPoint& ga = gp(0, u, fmax);
    const double gs = wk * P.uncertainty / ga.std;
    for (int f = 0; f < T; ++f)
      if (f == fmax)
        for (int i = 0; i < 3; ++i) g_a[f][i] += gs * ga.gstd[i];
  }
  // force cost
  double g_fn[NTA], g_sm[NTA];
  double gsm_dot = 0.0;
  for (int f = 0; f < T; ++f) {
    const double gv = v[f] <= 10.0 ? -wk : 0.0;
    g_fn[f] = gv * sm[f];
    g_sm[f] = gv * fn[f];
    gsm_dot += g_sm[f] * sm[f];
  }
  for (int f = 0; f < T; ++f) g_fn[f] += -(sm[f] * (g_sm[f] - gsm_dot));
  // contact margin reward (gain −200·wk)
  const double g_cr = -200.0 * wk;
  for (int f = 0; f < T; ++f) {
    double cdir[3], cdn, cang;
    contact(f, cdir, cdn, cang);
    const double gcang = g_cr * (0.1 / (cang + 1) + 0.9 / (cang - cos_mu + 1));
    double gdir[3] = {gcang * fe.n[f][0], gcang * fe.n[f][1], gcang * fe.n[f][2]};
    const double pd = dot3(cdir, gdir);
    for (int i = 0; i < 3; ++i) {
      const double gcd = (gdir[i] - cdir[i] * pd) / cdn;
      g_a[f][i] += gcd;
      o.g_target[f][i] -= gcd;
    }
  }
  // force_eq reward (gain −200·wk) + force norms
  fe.backward(-200.0 * wk, g_fn, in.comp, g_a, o.g_target, o.g_comp);
  // all-tip interpolation a = target + c·(tip − target)
  for (int f = 0; f < T; ++f) {
    const double c = (double)P.coeff[k][f];
    for (int i = 0; i < 3; ++i) {
      o.g_tip[f][i] = c * g_a[f][i];
      o.g_target[f][i] += g_a[f][i] - c * g_a[f][i];
    }
  }
}

// Forward + backward of Σ_levels w_k·l_k − 5·Σ pre_dist + 1/palm_dist for one candidate.
// gp(kind, level_or_0, finger) returns the GPIS results at the corresponding query.
template <typename GpisAt>
CDX_HD void closure_candidate(const cdx_problem& P, const CandidateIn& in, GpisAt gp, CandidateOut& out) {
  const int T = P.chain.n_tips;
  const int K = P.n_levels;
  double tip[CDX_MAX_TIPS][3];
  float tl[CDX_MAX_TIPS][3];
  double Rp[9];
  pregrasp_tips(P, in.q, in.palm_pos, in.palm_ori, tip, tl, Rp);

  double g_tip[CDX_MAX_TIPS][3];
  for (int f = 0; f < T; ++f) {
    g_tip[f][0] = g_tip[f][1] = g_tip[f][2] = 0.0;
    out.g_target[f][0] = out.g_target[f][1] = out.g_target[f][2] = 0.0;
    out.g_comp[f] = 0.0;
    out.margin[f] = 0.0;
  }
  for (int i = 0; i < P.chain.n_dofs; ++i) out.g_q[i] = 0.0;

  // ref_cost is identical on every level: ‖q − ref_q‖ with ref_q float32 (:732)
  double dq[CDX_MAX_DOFS];
  const double qnorm = ref_dist(P, in.q, dq);

  double total = 0.0;
  for (int k = 0; k < K; ++k) {
    const double wk = P.weight[k];
    LevelOut lo;
    level_fwd_bwd<0>(P, k, in, tip, qnorm, gp, lo);
    total += wk * lo.l;
    out.flip[k] = lo.flip;
    for (int f = 0; f < T; ++f) {
      out.margin[f] += wk * lo.margin[f];
      out.g_comp[f] += lo.g_comp[f];
      for (int i = 0; i < 3; ++i) { g_tip[f][i] += lo.g_tip[f][i]; out.g_target[f][i] += lo.g_target[f][i]; }
    }
    if (qnorm > 0)
      for (int i = 0; i < P.chain.n_dofs; ++i) out.g_q[i] += wk * 10.0 * dq[i] / qnorm;
  }
  // pregrasp-distance and palm-distance terms
  for (int f = 0; f < T; ++f) {
    const GpisPoint& gpp = gp(2, 0, f);
    for (int i = 0; i < 3; ++i) g_tip[f][i] += -5.0 * gpp.gmean[i];
  }
  double pre_sum = 0.0;
  for (int f = 0; f < T; ++f) pre_sum += gp(2, 0, f).mean;
  total = total - pre_sum * 5.0;
  for (int i = 0; i < 3; ++i) out.g_palm_pos[i] = 0.0;
  if (P.optimize_palm) {
    const GpisPoint& gpm = gp(3, 0, 0);
    total = total + 1.0 / gpm.mean;
    const double g = -1.0 / (gpm.mean * gpm.mean);
    for (int i = 0; i < 3; ++i) out.g_palm_pos[i] += g * gpm.gmean[i];
  }
  out.loss = total;
  // tip = Rp·tl + palm_pos
  double gRp[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  float gtl[CDX_MAX_TIPS * 3];
  for (int f = 0; f < T; ++f) {
    for (int i = 0; i < 3; ++i) out.g_palm_pos[i] += g_tip[f][i];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) gRp[3 * r + c] += g_tip[f][r] * (double)tl[f][c];
    double gl[3];
    mat3t_vec(Rp, g_tip[f], gl);
    for (int i = 0; i < 3; ++i) gtl[3 * f + i] = (float)gl[i];
  }
  double R_[9], dRa[9], dRb[9], dRc[9];
  euler_xyz(in.palm_ori, R_, dRa, dRb, dRc);
  out.g_palm_ori[0] = out.g_palm_ori[1] = out.g_palm_ori[2] = 0.0;
  for (int i = 0; i < 9; ++i) {
    out.g_palm_ori[0] += gRp[i] * dRa[i];
    out.g_palm_ori[1] += gRp[i] * dRb[i];
    out.g_palm_ori[2] += gRp[i] * dRc[i];
  }
  // FK backward in float32, then cast (q.float() backward)
  float qf[CDX_MAX_DOFS], gqf[CDX_MAX_DOFS];
  for (int i = 0; i < P.chain.n_dofs; ++i) { qf[i] = (float)in.q[i]; gqf[i] = 0.f; }
  for (int f = 0; f < T; ++f) fk_tip_bwd(P.chain, f, qf, &gtl[3 * f], GqAdd{gqf});
  for (int i = 0; i < P.chain.n_dofs; ++i) out.g_q[i] += (double)gqf[i];
}

}  // namespace cdx
