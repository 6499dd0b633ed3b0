// Per-candidate collision loss and its gradient (optimize_pregrasp.py:671-701), f64 with the
// anchors from f32 FK like the reference (:674-676).  Shared by the gfx950 kernel and the
// host test build.
#pragma once
#include "cdx_cost.h"

namespace cdx {

CDX_HD void collision_candidate(const cdx_collision& C, const double* q, const double* pp, const double* po,
                                double& cost, double* g_q, double* g_pp, double* g_po) {
  const int A = C.chain.n_tips, D = C.chain.n_dofs;
  float qf[CDX_MAX_DOFS];
  for (int i = 0; i < D; ++i) qf[i] = (float)q[i];
  double Rp[9], dRa[9], dRb[9], dRc[9];
  euler_xyz(po, Rp, dRa, dRb, dRc);
  float tl[CDX_MAX_TIPS][3];
  double a[CDX_MAX_TIPS][3], ga[CDX_MAX_TIPS][3];
  for (int k = 0; k < A; ++k) {
    fk_tip(C.chain, k, qf, tl[k], nullptr);
    const double v[3] = {(double)tl[k][0], (double)tl[k][1], (double)tl[k][2]};
    double w[3];
    mat3_vec(Rp, v, w);
    for (int i = 0; i < 3; ++i) { a[k][i] = w[i] + pp[i]; ga[k][i] = 0.0; }
  }
  // pairwise 1/d below the threshold (:679-686)
  double pair_cost = 0.0;
  for (int p = 0; p < C.n_pairs; ++p) {
    const int l = C.pairs[p][0], r = C.pairs[p][1];
    const double d[3] = {a[l][0] - a[r][0], a[l][1] - a[r][1], a[l][2] - a[r][2]};
    const double dist = sqrt(dot3(d, d));
    if (dist < C.pair_threshold) {
      pair_cost += 1.0 / dist;
      const double s = -1.0 / (dist * dist) / dist;  // d(1/dist)/dd = −d/dist³
      for (int i = 0; i < 3; ++i) { ga[l][i] += s * d[i]; ga[r][i] -= s * d[i]; }
    }
  }
  // floor (1/z)·0.1 below floor_z (:688-691)
  double z_cost = 0.0;
  for (int k = 0; k < A; ++k) {
    const double z = a[k][2];
    if (z < C.floor_z) {
      z_cost += (1.0 / z) * 0.1;
      ga[k][2] += -0.1 / (z * z);
    }
  }
  double c = pair_cost + z_cost;
  for (int i = 0; i < 3; ++i) g_pp[i] = 0.0;
  // palm floor 1/z (:693-698)
  if (C.palm_term && pp[2] < C.floor_z) {
    c += 1.0 / pp[2];
    g_pp[2] += -1.0 / (pp[2] * pp[2]);
  }
  cost = c;
  // back through a = Rp·tl + pp and the f32 FK
  double gR[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  float gqf[CDX_MAX_DOFS];
  for (int i = 0; i < D; ++i) gqf[i] = 0.f;
  for (int k = 0; k < A; ++k) {
    for (int i = 0; i < 3; ++i) g_pp[i] += ga[k][i];
    for (int r = 0; r < 3; ++r)
      for (int s = 0; s < 3; ++s) gR[3 * r + s] += ga[k][r] * (double)tl[k][s];
    double gl[3];
    mat3t_vec(Rp, ga[k], gl);
    const float gtl[3] = {(float)gl[0], (float)gl[1], (float)gl[2]};
    fk_tip_bwd(C.chain, k, qf, gtl, GqAdd{gqf});
  }
  g_po[0] = g_po[1] = g_po[2] = 0.0;
  for (int i = 0; i < 9; ++i) {
    g_po[0] += gR[i] * dRa[i];
    g_po[1] += gR[i] * dRb[i];
    g_po[2] += gR[i] * dRc[i];
  }
  for (int i = 0; i < D; ++i) g_q[i] = (double)gqf[i];
}

}  // namespace cdx
