// Fingertip forward kinematics (float32) and its vector-Jacobian product.
//
// Forward follows the non-recursive path of the reference:
//   joint pose  Rj = F·A(sign·q), F = (Rz(yaw)·Ry(pitch))·Rx(roll)   rigid_body.py:130-157
//   world pose  R_i = R_p·Rj_i,  t_i = R_p·t_i + t_p                 robot_model.py:174-194,
//                                                                    spatial_vector_algebra.py:98-103
//   quaternion  xyzw from the 4×4 M = [R t; 0 1] with the trace branch
//               and scale 0.5/sqrt(tn·M33)                           spatial_vector_algebra.py:108-136
//   tip         t_L + quat_rotate(quat, offset)                       robot_model.py:256-262,
//                                                                    se3_so3_util.py:240-250
// Backward reproduces the reference autograd graph, including its one artifact: the
// quaternion scale goes through math.sqrt on a tensor and is therefore a CONSTANT for
// autograd, so d tip/dR only sees the un-normalised quaternion times that constant.
#pragma once
#include "cdx_hd.h"

namespace cdx {

// Rotation about a principal axis by th and its derivative (spatial_vector_algebra.py:14-53).
CDX_HD void axis_rot(int axis, float th, float* A, float* dA) {
  const float c = cdx_cosf(th), s = cdx_sinf(th);
  for (int i = 0; i < 9; ++i) { A[i] = 0.f; dA[i] = 0.f; }
  if (axis == 0) {
    A[0] = 1.f; A[4] = c; A[5] = -s; A[7] = s; A[8] = c;
    dA[4] = -s; dA[5] = -c; dA[7] = c; dA[8] = -s;
  } else if (axis == 1) {
    A[0] = c; A[2] = s; A[4] = 1.f; A[6] = -s; A[8] = c;
    dA[0] = -s; dA[2] = c; dA[6] = -c; dA[8] = -s;
  } else {
    A[0] = c; A[1] = -s; A[3] = s; A[4] = c; A[8] = 1.f;
    dA[0] = -s; dA[1] = -c; dA[3] = c; dA[4] = -s;
  }
}

// Longest root→tip path a chain may have (iiwa7_allegro: 13).
#define CDX_MAX_DEPTH 16

// Bodies on the path from the root's child down to `body` as a bit mask (root = body 0 is the
// identity pose).  Parents precede children (urdf.py enforces it, chain_ok re-checks it), so
// ascending bit order is root→tip order: the path is walked without a per-thread array, which
// on the GPU would live in scratch memory.
CDX_HD uint32_t chain_path_mask(const cdx_chain& c, int body) {
  uint32_t m = 0;
  for (int n = 0; body > 0 && n < CDX_MAX_DEPTH; ++n) {
    m |= 1u << body;
    body = c.bodies[body].parent;
  }
  return m;
}
CDX_HD int low_bit(uint32_t m) { return __builtin_ctz(m); }
CDX_HD int high_bit(uint32_t m) { return 31 - __builtin_clz(m); }
CDX_HD int path_depth(uint32_t m) { return __builtin_popcount(m); }

// Joint-angle readers: q[i] as float32 from a float row, or a double row cast like the
// reference's q.float() (no per-thread copy of the row).
struct QRowD {
  const double* p;
  CDX_HDM float operator[](int i) const { return (float)p[i]; }
};

template <class Q>
CDX_HD void joint_rot(const cdx_body& b, const Q& q, float* Rj) {
  if (b.dof < 0) {
    for (int i = 0; i < 9; ++i) Rj[i] = b.F[i];
    return;
  }
  float A[9], dA[9];
  axis_rot(b.axis, b.sign * q[b.dof], A, dA);
  mat3_mul(b.F, A, Rj);
}

// Quaternion (xyzw) of a rotation with the reference branch; returns the un-scaled
// components in raw[4], the detached scale, and the branch id (-1 = trace branch,
// else the pivot index i of the other branch).
CDX_HD int quat_raw(const float* R, float* raw, float* scale) {
  const float M33 = 1.f;
  const float t = ((R[0] + R[4]) + R[8]) + M33;
  float tn;
  int br;
  if (t > M33) {
    tn = t;
    raw[3] = tn;
    raw[2] = R[3] - R[1];
    raw[1] = R[2] - R[6];
    raw[0] = R[7] - R[5];
    br = -1;
  } else {
    int i = 0, j = 1, k = 2;
    if (R[4] > R[0]) { i = 1; j = 2; k = 0; }
    if (R[8] > R[4 * i]) { i = 2; j = 0; k = 1; }
    tn = R[4 * i] - (R[4 * j] + R[4 * k]) + M33;
    raw[i] = tn;
    raw[j] = R[3 * i + j] + R[3 * j + i];
    raw[k] = R[3 * k + i] + R[3 * i + k];
    raw[3] = R[3 * k + j] - R[3 * j + k];
    br = i;
  }
  *scale = (float)(0.5 / sqrt((double)(tn * M33)));
  return br;
}

// d raw / dR accumulated into gR given g_raw.
CDX_HD void quat_raw_bwd(int br, const float* g, float* gR) {
  if (br < 0) {
    gR[0] += g[3]; gR[4] += g[3]; gR[8] += g[3];
    gR[3] += g[2]; gR[1] -= g[2];
    gR[2] += g[1]; gR[6] -= g[1];
    gR[7] += g[0]; gR[5] -= g[0];
  } else {
    const int i = br, j = (br + 1) % 3, k = (br + 2) % 3;
    gR[4 * i] += g[i]; gR[4 * j] -= g[i]; gR[4 * k] -= g[i];
    gR[3 * i + j] += g[j]; gR[3 * j + i] += g[j];
    gR[3 * k + i] += g[k]; gR[3 * i + k] += g[k];
    gR[3 * k + j] += g[3]; gR[3 * j + k] -= g[3];
  }
}

// v(2w²−1) + 2w(q×v) + 2q(q·v)  (se3_so3_util.py:240-250)
CDX_HD void quat_rotate(const float* q, const float* v, float* out) {
  const float w = q[3];
  const float a = 2.0f * (w * w) - 1.0f;
  const float cx = q[1] * v[2] - q[2] * v[1];
  const float cy = q[2] * v[0] - q[0] * v[2];
  const float cz = q[0] * v[1] - q[1] * v[0];
  const float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  out[0] = v[0] * a + cx * w * 2.0f + q[0] * d * 2.0f;
  out[1] = v[1] * a + cy * w * 2.0f + q[1] * d * 2.0f;
  out[2] = v[2] * a + cz * w * 2.0f + q[2] * d * 2.0f;
}

// gq += ∂(G·quat_rotate(q,v))/∂q
CDX_HD void quat_rotate_bwd(const float* q, const float* v, const float* G, float* gq) {
  const float w = q[3];
  const float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  const float Gv = G[0] * v[0] + G[1] * v[1] + G[2] * v[2];
  const float Gq = G[0] * q[0] + G[1] * q[1] + G[2] * q[2];
  // G·(q×v) = q·(v×G)
  const float vxG0 = v[1] * G[2] - v[2] * G[1];
  const float vxG1 = v[2] * G[0] - v[0] * G[2];
  const float vxG2 = v[0] * G[1] - v[1] * G[0];
  const float Gqv = q[0] * vxG0 + q[1] * vxG1 + q[2] * vxG2;
  gq[3] += 4.0f * w * Gv + 2.0f * Gqv;
  gq[0] += 2.0f * w * vxG0 + 2.0f * (d * G[0] + Gq * v[0]);
  gq[1] += 2.0f * w * vxG1 + 2.0f * (d * G[1] + Gq * v[1]);
  gq[2] += 2.0f * w * vxG2 + 2.0f * (d * G[2] + Gq * v[2]);
}

// One step of the world-pose recurrence: t' = R·t_b + t, R' = R·Rj  (robot_model.py:174-194).
template <class Q>
CDX_HD void chain_step(const cdx_body& b, const Q& q, const float* R, const float* t, float* Rn, float* tn) {
  float Rj[9], tt[3];
  joint_rot(b, q, Rj);
  mat3_vec(R, b.t, tt);
  tn[0] = tt[0] + t[0];
  tn[1] = tt[1] + t[1];
  tn[2] = tt[2] + t[2];
  mat3_mul(R, Rj, Rn);
}

// Tip position (and quaternion) of tip `k` from the final pose (R, t) of its body.
CDX_HD void tip_from_pose(const cdx_chain& c, int k, const float* R, const float* t, float* pos, float* quat) {
  float raw[4], sc;
  quat_raw(R, raw, &sc);
  float qt[4] = {raw[0] * sc, raw[1] * sc, raw[2] * sc, raw[3] * sc};
  pos[0] = t[0]; pos[1] = t[1]; pos[2] = t[2];
  if (c.has_offsets) {
    float o[3];
    quat_rotate(qt, c.tip_offset[k], o);
    pos[0] = pos[0] + o[0]; pos[1] = pos[1] + o[1]; pos[2] = pos[2] + o[2];
  }
  if (quat) for (int i = 0; i < 4; ++i) quat[i] = qt[i];
}

// Tip position (and quaternion) of tip `k`: running pose, no per-level storage.
template <class Q>
CDX_HD void fk_tip(const cdx_chain& c, int k, const Q& q, float* pos, float* quat) {
  float R[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f}, t[3] = {0.f, 0.f, 0.f};
  for (uint32_t m = chain_path_mask(c, c.tip_body[k]); m; m &= m - 1) {
    float Rn[9], tn[3];
    chain_step(c.bodies[low_bit(m)], q, R, t, Rn, tn);
    for (int i = 0; i < 9; ++i) R[i] = Rn[i];
    for (int i = 0; i < 3; ++i) t[i] = tn[i];
  }
  tip_from_pose(c, k, R, t, pos, quat);
}

// g_q(dof, v) receives (∂pos_k/∂q)ᵀ·gpos, one call per moving joint on the path, with the
// reference's gradient semantics; pos (nullable) receives the tip position.  The parent poses
// the backward needs are kept in a register array of MAXD levels (loops unrolled over the
// bound, guarded by the path depth): MAXD must cover the chain's deepest tip (see
// chain_max_depth); CDX_MAX_DEPTH covers every chain.
template <int MAXD = CDX_MAX_DEPTH, class Q, class GQ>
CDX_HD void fk_tip_bwd(const cdx_chain& c, int k, const Q& q, const float* gpos, GQ&& g_q, float* pos = nullptr) {
  const uint32_t mask = chain_path_mask(c, c.tip_body[k]);
  const int n = path_depth(mask);
  float Rs[MAXD][9];  // Rs[l]: world rotation of level l's parent
  float R[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f}, t[3] = {0.f, 0.f, 0.f};
  uint32_t m = mask;
#pragma unroll
  for (int l = 0; l < MAXD; ++l) {
    if (l < n) {
      for (int i = 0; i < 9; ++i) Rs[l][i] = R[i];
      float Rn[9], tn[3];
      chain_step(c.bodies[low_bit(m)], q, R, t, Rn, tn);
      m &= m - 1;
      for (int i = 0; i < 9; ++i) R[i] = Rn[i];
      for (int i = 0; i < 3; ++i) t[i] = tn[i];
    }
  }
  if (pos) tip_from_pose(c, k, R, t, pos, nullptr);
  float GR[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  float Gt[3] = {gpos[0], gpos[1], gpos[2]};
  if (c.has_offsets) {
    float raw[4], sc;
    const int br = quat_raw(R, raw, &sc);
    float qt[4] = {raw[0] * sc, raw[1] * sc, raw[2] * sc, raw[3] * sc};
    float gq[4] = {0, 0, 0, 0};
    quat_rotate_bwd(qt, c.tip_offset[k], gpos, gq);
    for (int i = 0; i < 4; ++i) gq[i] *= sc;  // scale is detached: only d raw flows
    quat_raw_bwd(br, gq, GR);
  }
  m = mask;
#pragma unroll
  for (int l = MAXD - 1; l >= 0; --l) {
    if (l < n) {
      const int bi = high_bit(m);
      m &= ~(1u << bi);
      const cdx_body& b = c.bodies[bi];
      float Rj[9], A[9], dA[9];
      if (b.dof >= 0) {
        axis_rot(b.axis, b.sign * q[b.dof], A, dA);
        mat3_mul(b.F, A, Rj);
        // G_Rj = R_pᵀ·G_R ;  G_A = Fᵀ·G_Rj ; dθ = <G_A, dA>
        float GRj[9], GA[9];
        mat3_mul_tn(Rs[l], GR, GRj);
        mat3_mul_tn(b.F, GRj, GA);
        float dth = 0.f;
        for (int i = 0; i < 9; ++i) dth += GA[i] * dA[i];
        g_q(b.dof, b.sign * dth);
      } else {
        for (int i = 0; i < 9; ++i) Rj[i] = b.F[i];
      }
      // G_R_p = G_R·Rjᵀ + G_t ⊗ t_b ;  G_t_p = G_t
      float GRp[9];
      mat3_mul_nt(GR, Rj, GRp);
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) GRp[3 * i + j] += Gt[i] * b.t[j];
      for (int i = 0; i < 9; ++i) GR[i] = GRp[i];
    }
  }
}

// fk_tip_bwd in closed form, no per-level storage: every joint is a revolute joint about a body axis (axis_rot)
// or fixed, so with M_j = R_parent·F_j (orthonormal), ω_j = M_j·e_axis and o_j the joint's world origin,
// dR/dθ_j = [ω_j]×R and dt/dθ_j = ω_j × (t − o_j) for the final pose (R, t).  Hence
//   dL/dθ_j = <G_R, [ω_j]×R> + G_t·(ω_j × (t − o_j)) = ω_j·(w − o_j × G_t),  w = Σ_c R[:,c] × G_R[:,c] + t × G_t,
// with G_R the tip offset's rotation gradient (the detached-scale quaternion path as in fk_tip_bwd).  Two forward
// walks (the second recomputes the poses) instead of a forward walk that keeps every level's rotation plus a
// backward walk: the same gradient to f32 rounding, ≈ 10 registers of state instead of 9 per level.
template <int MAXD, class Q, class GQ>
CDX_HD void fk_tip_bwd2(const cdx_chain& c, int k, const Q& q, const float* gpos, GQ&& g_q, float* pos = nullptr) {
  const uint32_t mask = chain_path_mask(c, c.tip_body[k]);
  const int n = path_depth(mask);
  float R[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f}, t[3] = {0.f, 0.f, 0.f};
  uint32_t m = mask;
#pragma unroll
  for (int l = 0; l < MAXD; ++l) {
    if (l < n) {
      float Rn[9], tn[3];
      chain_step(c.bodies[low_bit(m)], q, R, t, Rn, tn);
      m &= m - 1;
      for (int i = 0; i < 9; ++i) R[i] = Rn[i];
      for (int i = 0; i < 3; ++i) t[i] = tn[i];
    }
  }
  if (pos) tip_from_pose(c, k, R, t, pos, nullptr);
  float GR[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const float Gt[3] = {gpos[0], gpos[1], gpos[2]};
  if (c.has_offsets) {
    float raw[4], sc;
    const int br = quat_raw(R, raw, &sc);
    float qt[4] = {raw[0] * sc, raw[1] * sc, raw[2] * sc, raw[3] * sc};
    float gq[4] = {0, 0, 0, 0};
    quat_rotate_bwd(qt, c.tip_offset[k], gpos, gq);
    for (int i = 0; i < 4; ++i) gq[i] *= sc;  // scale is detached: only d raw flows
    quat_raw_bwd(br, gq, GR);
  }
  float w[3] = {t[1] * Gt[2] - t[2] * Gt[1], t[2] * Gt[0] - t[0] * Gt[2], t[0] * Gt[1] - t[1] * Gt[0]};
#pragma unroll
  for (int cc = 0; cc < 3; ++cc) {
    const float r0 = R[cc], r1 = R[3 + cc], r2 = R[6 + cc], g0 = GR[cc], g1 = GR[3 + cc], g2 = GR[6 + cc];
    w[0] += r1 * g2 - r2 * g1;
    w[1] += r2 * g0 - r0 * g2;
    w[2] += r0 * g1 - r1 * g0;
  }
  for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.f : 0.f;
  t[0] = t[1] = t[2] = 0.f;
  m = mask;
#pragma unroll
  for (int l = 0; l < MAXD; ++l) {
    if (l < n) {
      const cdx_body& b = c.bodies[low_bit(m)];
      m &= m - 1;
      float M[9], tt[3];
      mat3_mul(R, b.F, M);
      mat3_vec(R, b.t, tt);
      for (int i = 0; i < 3; ++i) t[i] = tt[i] + t[i];
      if (b.dof >= 0) {
        const int ax = b.axis;  // (selects, not an index into M: a register array indexed at run time goes to scratch)
        const float om[3] = {ax == 0 ? M[0] : (ax == 1 ? M[1] : M[2]), ax == 0 ? M[3] : (ax == 1 ? M[4] : M[5]),
                             ax == 0 ? M[6] : (ax == 1 ? M[7] : M[8])};
        const float ox[3] = {t[1] * Gt[2] - t[2] * Gt[1], t[2] * Gt[0] - t[0] * Gt[2], t[0] * Gt[1] - t[1] * Gt[0]};
        const float dth = om[0] * (w[0] - ox[0]) + om[1] * (w[1] - ox[1]) + om[2] * (w[2] - ox[2]);
        g_q(b.dof, b.sign * dth);
        float A[9], dA[9];
        axis_rot(b.axis, b.sign * q[b.dof], A, dA);
        mat3_mul(M, A, R);
      } else {
        for (int i = 0; i < 9; ++i) R[i] = M[i];
      }
    }
  }
}

// fk_tip_bwd2's gradient from ONE walk: each moving joint's world axis ω_j = R_parent·F_j·e_axis and origin o_j are kept
// (6 floats per level, MAXD levels in registers) during the forward walk, and dθ_j = ω_j·(w − o_j × G_t) is taken for
// every joint once w is known — no second walk (its sin / cos and matrix products), and the per-joint products are
// independent of each other.  For shallow chains (MAXD ≤ 8: the hands), where the registers are affordable.
template <int MAXD, class Q, class GQ>
CDX_HD void fk_tip_bwd3(const cdx_chain& c, int k, const Q& q, const float* gpos, GQ&& g_q, float* pos = nullptr) {
  const uint32_t mask = chain_path_mask(c, c.tip_body[k]);
  const int n = path_depth(mask);
  float R[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f}, t[3] = {0.f, 0.f, 0.f};
  float om[MAXD][3], og[MAXD][3], sgn[MAXD];
  int dof[MAXD];
  uint32_t m = mask;
#pragma unroll
  for (int l = 0; l < MAXD; ++l) {
    dof[l] = -1;
    if (l < n) {
      const cdx_body& b = c.bodies[low_bit(m)];
      m &= m - 1;
      float Rn[9], tn[3];
      chain_step(b, q, R, t, Rn, tn);
      if (b.dof >= 0) {
        const int ax = b.axis;  // (selects: a register array indexed at run time goes to scratch)
        const float fa[3] = {ax == 0 ? b.F[0] : (ax == 1 ? b.F[1] : b.F[2]), ax == 0 ? b.F[3] : (ax == 1 ? b.F[4] : b.F[5]),
                             ax == 0 ? b.F[6] : (ax == 1 ? b.F[7] : b.F[8])};
        mat3_vec(R, fa, om[l]);
        for (int i = 0; i < 3; ++i) og[l][i] = tn[i];
        dof[l] = b.dof;
        sgn[l] = b.sign;
      }
      for (int i = 0; i < 9; ++i) R[i] = Rn[i];
      for (int i = 0; i < 3; ++i) t[i] = tn[i];
    }
  }
  if (pos) tip_from_pose(c, k, R, t, pos, nullptr);
  float GR[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const float Gt[3] = {gpos[0], gpos[1], gpos[2]};
  if (c.has_offsets) {
    float raw[4], sc;
    const int br = quat_raw(R, raw, &sc);
    float qt[4] = {raw[0] * sc, raw[1] * sc, raw[2] * sc, raw[3] * sc};
    float gq[4] = {0, 0, 0, 0};
    quat_rotate_bwd(qt, c.tip_offset[k], gpos, gq);
    for (int i = 0; i < 4; ++i) gq[i] *= sc;  // scale is detached: only d raw flows
    quat_raw_bwd(br, gq, GR);
  }
  float w[3] = {t[1] * Gt[2] - t[2] * Gt[1], t[2] * Gt[0] - t[0] * Gt[2], t[0] * Gt[1] - t[1] * Gt[0]};
#pragma unroll
  for (int cc = 0; cc < 3; ++cc) {
    const float r0 = R[cc], r1 = R[3 + cc], r2 = R[6 + cc], g0 = GR[cc], g1 = GR[3 + cc], g2 = GR[6 + cc];
    w[0] += r1 * g2 - r2 * g1;
    w[1] += r2 * g0 - r0 * g2;
    w[2] += r0 * g1 - r1 * g0;
  }
#pragma unroll
  for (int l = 0; l < MAXD; ++l) {
    if (dof[l] >= 0) {
      const float* o = og[l];
      const float ox[3] = {o[1] * Gt[2] - o[2] * Gt[1], o[2] * Gt[0] - o[0] * Gt[2], o[0] * Gt[1] - o[1] * Gt[0]};
      const float dth = om[l][0] * (w[0] - ox[0]) + om[l][1] * (w[1] - ox[1]) + om[l][2] * (w[2] - ox[2]);
      g_q(dof[l], sgn[l] * dth);
    }
  }
}

// fk_tip_bwd3 with the joints' axes and origins in caller-provided memory instead of registers (deep chains, where the
// registers are spent), in its two halves, so that a walk done earlier (the fused Kin iteration's next-fingertip FK,
// which walks the same joint row) can stand in for the first: fk_tip_walk3s leaves the final pose and, through
// put(l, i, v), each moving joint's slots at path level l (i < 3: ω, 3 ≤ i < 6: o); fk_tip_bwd3_grad takes the
// per-joint products from get(l, i).  Rolled loops over the path: the unrolled form (MAXD copies of the joint's
// sin / cos and products) measured ≈ 1.7× the cycles of a walk at one wave per SIMD, kin_cost4_kernel's occupancy
// (tools/kin_phases.py).
template <class Q, class PUT>
CDX_HD void fk_tip_walk3s(const cdx_chain& c, int k, const Q& q, float* R, float* t, PUT&& put) {
  for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.f : 0.f;
  t[0] = t[1] = t[2] = 0.f;
  int l = 0;
  for (uint32_t m = chain_path_mask(c, c.tip_body[k]); m; m &= m - 1, ++l) {
    const cdx_body& b = c.bodies[low_bit(m)];
    float Rn[9], tn[3];
    chain_step(b, q, R, t, Rn, tn);
    if (b.dof >= 0) {
      const int ax = b.axis;
      const float fa[3] = {ax == 0 ? b.F[0] : (ax == 1 ? b.F[1] : b.F[2]), ax == 0 ? b.F[3] : (ax == 1 ? b.F[4] : b.F[5]),
                           ax == 0 ? b.F[6] : (ax == 1 ? b.F[7] : b.F[8])};
      float om[3];
      mat3_vec(R, fa, om);
      for (int i = 0; i < 3; ++i) {
        put(l, i, om[i]);
        put(l, 3 + i, tn[i]);
      }
    }
    for (int i = 0; i < 9; ++i) R[i] = Rn[i];
    for (int i = 0; i < 3; ++i) t[i] = tn[i];
  }
}

template <class GQ, class GET>
CDX_HD void fk_tip_bwd3_grad(const cdx_chain& c, int k, const float* R, const float* t, const float* gpos, GQ&& g_q,
                             GET&& get) {
  float GR[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const float Gt[3] = {gpos[0], gpos[1], gpos[2]};
  if (c.has_offsets) {
    float raw[4], sc;
    const int br = quat_raw(R, raw, &sc);
    float qt[4] = {raw[0] * sc, raw[1] * sc, raw[2] * sc, raw[3] * sc};
    float gq[4] = {0, 0, 0, 0};
    quat_rotate_bwd(qt, c.tip_offset[k], gpos, gq);
    for (int i = 0; i < 4; ++i) gq[i] *= sc;  // scale is detached: only d raw flows
    quat_raw_bwd(br, gq, GR);
  }
  float w[3] = {t[1] * Gt[2] - t[2] * Gt[1], t[2] * Gt[0] - t[0] * Gt[2], t[0] * Gt[1] - t[1] * Gt[0]};
#pragma unroll
  for (int cc = 0; cc < 3; ++cc) {
    const float r0 = R[cc], r1 = R[3 + cc], r2 = R[6 + cc], g0 = GR[cc], g1 = GR[3 + cc], g2 = GR[6 + cc];
    w[0] += r1 * g2 - r2 * g1;
    w[1] += r2 * g0 - r0 * g2;
    w[2] += r0 * g1 - r1 * g0;
  }
  int l = 0;
  for (uint32_t m = chain_path_mask(c, c.tip_body[k]); m; m &= m - 1, ++l) {
    const cdx_body& b = c.bodies[low_bit(m)];
    if (b.dof >= 0) {
      float om[3], o[3];
      for (int i = 0; i < 3; ++i) {
        om[i] = get(l, i);
        o[i] = get(l, 3 + i);
      }
      const float ox[3] = {o[1] * Gt[2] - o[2] * Gt[1], o[2] * Gt[0] - o[0] * Gt[2], o[0] * Gt[1] - o[1] * Gt[0]};
      const float dth = om[0] * (w[0] - ox[0]) + om[1] * (w[1] - ox[1]) + om[2] * (w[2] - ox[2]);
      g_q(b.dof, b.sign * dth);
    }
  }
}

// Deepest tip path of a chain (host: picks the fk_tip_bwd register bound).
CDX_HD int chain_max_depth(const cdx_chain& c) {
  int d = 0;
  for (int k = 0; k < c.n_tips; ++k) {
    const int n = path_depth(chain_path_mask(c, c.tip_body[k]));
    d = n > d ? n : d;
  }
  return d;
}

// Array accumulator for fk_tip_bwd: g[dof] += v.
struct GqAdd {
  float* g;
  CDX_HDM void operator()(int d, float v) const { g[d] += v; }
};

}  // namespace cdx
