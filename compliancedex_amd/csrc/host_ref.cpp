// Host (x86) build of the per-candidate device code in cdx_fk.h / cdx_cost.h / cdx_collision.h /
// cdx_sdf.h.
//
// TEST-ONLY: libcdx_host.so lets the CPU test suite check the hand-derived backward
// (Kabsch/SVD, cost terms, FK) against the oracle's autograd without a GPU.  The
// product path never loads it; the Python package loads only the gfx950 libcdx.so.
#include <string.h>

#include "cdx_collision.h"
#include "cdx_cost.h"
#include "cdx_sdf.h"

namespace {

struct HostGpis {
  const double *mean, *gmean, *normal, *std_, *gstd;
  int64_t E, e;
  int T, Lq;
  cdx::GpisPoint operator()(int kind, int u, int f) const {
    cdx::GpisPoint p;
    int64_t qi;
    if (kind == 0) qi = cdx::q_alltip(u, e, f, E, T);
    else if (kind == 1) qi = cdx::q_target(Lq, e, f, E, T);
    else if (kind == 2) qi = cdx::q_pre(Lq, e, f, E, T);
    else qi = cdx::q_palm(Lq, e, E, T);
    memset(&p, 0, sizeof(p));
    p.mean = mean[qi];
    for (int i = 0; i < 3; ++i) p.gmean[i] = gmean[3 * qi + i];
    if (kind == 0) {
      p.std = std_[qi];
      for (int i = 0; i < 3; ++i) { p.gstd[i] = gstd[3 * qi + i]; p.normal[i] = normal[3 * qi + i]; }
    }
    return p;
  }
};

}  // namespace

extern "C" {

void cdxh_fk_forward(const cdx_chain* c, const float* q, int64_t B, float* pos, float* quat) {
  for (int64_t b = 0; b < B; ++b)
    for (int k = 0; k < c->n_tips; ++k)
      cdx::fk_tip(*c, k, q + b * c->n_dofs, pos + (b * c->n_tips + k) * 3, quat ? quat + (b * c->n_tips + k) * 4 : nullptr);
}

void cdxh_fk_backward(const cdx_chain* c, const float* q, int64_t B, const float* gpos, float* gq) {
  for (int64_t b = 0; b < B; ++b) {
    float* g = gq + b * c->n_dofs;
    for (int i = 0; i < c->n_dofs; ++i) g[i] = 0.f;
    for (int k = 0; k < c->n_tips; ++k) cdx::fk_tip_bwd(*c, k, q + b * c->n_dofs, gpos + (b * c->n_tips + k) * 3, cdx::GqAdd{g});
  }
}

int64_t cdxh_n_queries(const cdx_problem* P, int64_t E) { return cdx::n_queries(*P, E); }

void cdxh_closure_queries(const cdx_problem* P, int64_t E, const double* q, const double* target, const double* palm_pos,
                          const double* palm_ori, double* X) {
  const int T = P->chain.n_tips, D = P->chain.n_dofs, Lq = P->n_query_levels;
  for (int64_t e = 0; e < E; ++e) {
    double tip[CDX_MAX_TIPS][3], Rp[9];
    float tl[CDX_MAX_TIPS][3];
    cdx::pregrasp_tips(*P, q + e * D, palm_pos + 3 * e, palm_ori + 3 * e, tip, tl, Rp);
    const double* tg = target + e * T * 3;
    for (int u = 0; u < Lq; ++u) {
      int k = 0;
      while (k < P->n_levels - 1 && P->level_query[k] != u) ++k;
      for (int f = 0; f < T; ++f) {
        const double c = (double)P->coeff[k][f];
        const int64_t qi = cdx::q_alltip(u, e, f, E, T);
        for (int i = 0; i < 3; ++i) X[3 * qi + i] = tg[3 * f + i] + c * (tip[f][i] - tg[3 * f + i]);
      }
    }
    for (int f = 0; f < T; ++f)
      for (int i = 0; i < 3; ++i) {
        X[3 * cdx::q_target(Lq, e, f, E, T) + i] = tg[3 * f + i];
        X[3 * cdx::q_pre(Lq, e, f, E, T) + i] = tip[f][i];
      }
    if (P->optimize_palm)
      for (int i = 0; i < 3; ++i) X[3 * cdx::q_palm(Lq, e, E, T) + i] = palm_pos[3 * e + i];
  }
}

void cdxh_closure_cost(const cdx_problem* P, int64_t E, const double* q, const double* comp, const double* target,
                       const double* palm_pos, const double* palm_ori, const double* noise, const double* mean,
                       const double* gmean, const double* normal, const double* std_, const double* gstd,
                       double* total_loss, double* total_margin, double* g_q, double* g_comp, double* g_target,
                       double* g_palm_pos, double* g_palm_ori, int32_t* flip) {
  const int T = P->chain.n_tips, D = P->chain.n_dofs;
  HostGpis g{mean, gmean, normal, std_, gstd, E, 0, T, P->n_query_levels};
  for (int64_t e = 0; e < E; ++e) {
    cdx::CandidateIn in;
    in.q = q + e * D;
    in.comp = comp + e * T;
    in.target = target + e * T * 3;
    in.palm_pos = palm_pos + 3 * e;
    in.palm_ori = palm_ori + 3 * e;
    in.noise = noise + e * 9;
    in.noise_stride = E * 9;
    g.e = e;
    cdx::CandidateOut out;
    cdx::closure_candidate(*P, in, g, out);
    total_loss[e] = out.loss;
    for (int f = 0; f < T; ++f) {
      total_margin[e * T + f] = out.margin[f];
      g_comp[e * T + f] = out.g_comp[f];
      for (int i = 0; i < 3; ++i) g_target[(e * T + f) * 3 + i] = out.g_target[f][i];
    }
    for (int i = 0; i < D; ++i) g_q[e * D + i] = out.g_q[i];
    for (int i = 0; i < 3; ++i) { g_palm_pos[3 * e + i] = out.g_palm_pos[i]; g_palm_ori[3 * e + i] = out.g_palm_ori[i]; }
    for (int k = 0; k < P->n_levels; ++k) flip[k * E + e] = out.flip[k];
  }
}

void cdxh_collision(const cdx_collision* C, int64_t E, const double* q, const double* pp, const double* po,
                    double* cost, double* g_q, double* g_pp, double* g_po) {
  const int D = C->chain.n_dofs;
  for (int64_t e = 0; e < E; ++e)
    cdx::collision_candidate(*C, q + e * D, pp + 3 * e, po + 3 * e, cost[e], g_q + e * D, g_pp + 3 * e, g_po + 3 * e);
}

void cdxh_force_eq(const cdx_force_eq* p, int64_t B, const double* tip, const double* target, const double* comp,
                   const double* normal, const double* noise, const double* g_reward, const double* g_fn,
                   double* reward, double* margin, double* fn, int32_t* flip, double* g_tip, double* g_target,
                   double* g_comp) {
  cdx::ForceEqParams fp;
  fp.cos_mu = (double)p->cos_mu;
  fp.gravity = p->gravity;
  for (int i = 0; i < 3; ++i) fp.com[i] = (double)p->com[i];
  fp.dummy_target_z = (double)p->dummy_target_z;
  fp.dummy_comp = (double)p->dummy_comp;
  const int T = p->n_tips;
  for (int64_t b = 0; b < B; ++b) {
    double tp[CDX_MAX_TIPS][3], nr[CDX_MAX_TIPS][3];
    for (int f = 0; f < T; ++f)
      for (int i = 0; i < 3; ++i) { tp[f][i] = tip[(b * T + f) * 3 + i]; nr[f][i] = normal[(b * T + f) * 3 + i]; }
    cdx::ForceEq<0> fe;
    fe.forward(fp, T, tp, target + b * T * 3, comp + b * T, nr, noise + b * 9);
    reward[b] = fe.reward;
    flip[b] = fe.flip;
    double gt[CDX_MAX_TIPS][3] = {}, gg[CDX_MAX_TIPS][3] = {}, gc[CDX_MAX_TIPS] = {};
    for (int f = 0; f < T; ++f) { margin[b * T + f] = fe.margin[f]; fn[b * T + f] = fe.fn[f]; }
    fe.backward(g_reward[b], g_fn + b * T, comp + b * T, gt, gg, gc);
    for (int f = 0; f < T; ++f) {
      for (int i = 0; i < 3; ++i) { g_tip[(b * T + f) * 3 + i] = gt[f][i]; g_target[(b * T + f) * 3 + i] = gg[f][i]; }
      g_comp[b * T + f] = gc[f];
    }
  }
}

void cdxh_svd3(const double* H, double* U, double* S, double* V) { cdx::svd3(H, U, S, V); }

void cdxh_sdf_forward(const float* points, int64_t P, const float* faces, int64_t F, float* dist, int32_t* sign,
                      float* nrm, float* clst, int32_t* face) {
  for (int64_t i = 0; i < P; ++i) {
    const cdx::F3 p = cdx::f3(points[3 * i], points[3 * i + 1], points[3 * i + 2]);
    float best = 0;
    int bs = 0, bf = -1;
    cdx::F3 bn = cdx::f3(0, 0, 0), bc = bn;
    for (int64_t f0 = 0; f0 < F; f0 += CDX_SDF_REF_TILE) {
      const int64_t nt = F - f0 < CDX_SDF_REF_TILE ? F - f0 : CDX_SDF_REF_TILE;
      float tb = 0;
      int ts = 0, tf = -1;
      cdx::F3 tn = bn, tc = bn;
      for (int64_t s = 0; s < nt; ++s) {
        const float* v = faces + 9 * (f0 + s);
        cdx::F3 c, n;
        int sg;
        const float d = cdx::point_face(p, cdx::f3(v[0], v[1], v[2]), cdx::f3(v[3], v[4], v[5]), cdx::f3(v[6], v[7], v[8]), c, n, sg);
        if (s == 0 || tb > d) { tb = d; ts = sg; tn = n; tc = c; tf = (int)(f0 + s); }
      }
      if (f0 == 0 || best > tb) { best = tb; bs = ts; bn = tn; bc = tc; bf = tf; }
    }
    dist[i] = best;
    sign[i] = bs;
    nrm[3 * i] = bn.x; nrm[3 * i + 1] = bn.y; nrm[3 * i + 2] = bn.z;
    clst[3 * i] = bc.x; clst[3 * i + 1] = bc.y; clst[3 * i + 2] = bc.z;
    if (face) face[i] = bf;
  }
}

// Test-only: face_dist2 (the culled kernels' evaluation from a face record) and point_face's squared
// distance for n (point, face) pairs — tests/test_sdf_cpu.py checks them bit-identical.
void cdxh_face_dist2(const float* points, const float* faces, int64_t n, float* d_rec, float* d_ref) {
  for (int64_t i = 0; i < n; ++i) {
    const cdx::F3 p = cdx::f3(points[3 * i], points[3 * i + 1], points[3 * i + 2]);
    const float* v = faces + 9 * i;
    const cdx::F3 v1 = cdx::f3(v[0], v[1], v[2]), v2 = cdx::f3(v[3], v[4], v[5]), v3 = cdx::f3(v[6], v[7], v[8]);
    d_rec[i] = cdx::face_dist2(p, cdx::face_rec(v1, v2, v3, (int)i));
    cdx::F3 c, nrm;
    int sg;
    d_ref[i] = cdx::point_face(p, v1, v2, v3, c, nrm, sg);
  }
}

}  // extern "C"
