// Fused optimizer step for the prob-mode loop (optimize_pregrasp.py:805-836): one thread per
// candidate; best-iterate update, Adam on the five parameter groups, clamps.  Float64 like the
// reference parameters.
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/cdx.h"

namespace {

struct AdamScalars {
  double beta1, beta2, eps, step_size, bc2_sqrt;
};

// torch.optim.Adam single-tensor / foreach order (torch/optim/adam.py)
__device__ __forceinline__ double adam_update(double p, double g, double& m, double& v, const AdamScalars& a) {
  m = m + (1.0 - a.beta1) * (g - m);          // lerp_(g, 1-β1), weight < 0.5 branch
  v = v * a.beta2 + ((1.0 - a.beta2) * g) * g; // mul_(β2).addcmul_(g, g, 1-β2)
  const double denom = sqrt(v) / a.bc2_sqrt + a.eps;
  return p + (a.step_size * m) / denom;        // addcdiv_(m, denom, value=-lr/bc1)
}

__global__ __launch_bounds__(64) void optimizer_step_kernel(cdx_adam cfg, cdx_opt_buffers b, int64_t E, int D, int T,
                                                            int s) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  if (b.loop) s = b.loop->step;  // graph-replayable loop: the closure advanced it
  // best iterate (before the step, with the parameters the closure saw)
  if (s > cfg.best_after && b.total_loss[e] < b.opt_value[e]) {
    b.opt_value[e] = b.total_loss[e];
    for (int f = 0; f < T; ++f) {
      b.opt_margin[e * T + f] = b.total_margin[e * T + f];
      b.opt_comp[e * T + f] = b.comp[e * T + f];
      for (int i = 0; i < 3; ++i) b.opt_target[(e * T + f) * 3 + i] = b.target[(e * T + f) * 3 + i];
    }
    for (int i = 0; i < D; ++i) b.opt_q[e * D + i] = b.q[e * D + i];
    for (int i = 0; i < 3; ++i) { b.opt_palm[6 * e + i] = b.palm_pos[3 * e + i]; b.opt_palm[6 * e + 3 + i] = b.palm_ori[3 * e + i]; }
  }
  const double t = (double)(s + 1);
  const double bc1 = 1.0 - pow(cfg.beta1, t), bc2 = 1.0 - pow(cfg.beta2, t);
  AdamScalars a;
  a.beta1 = cfg.beta1; a.beta2 = cfg.beta2; a.eps = cfg.eps; a.bc2_sqrt = sqrt(bc2);
  // group 0: joint angles
  if (cfg.lr[0] != 0.0) {
    a.step_size = -(cfg.lr[0] / bc1);
    for (int i = 0; i < D; ++i) {
      const int64_t k = e * D + i;
      b.q[k] = adam_update(b.q[k], b.g_q[k], b.m_q[k], b.v_q[k], a);
    }
  }
  // group 1: compliance, then clamp_(min=comp_min)
  if (cfg.lr[1] != 0.0) {
    a.step_size = -(cfg.lr[1] / bc1);
    for (int f = 0; f < T; ++f) {
      const int64_t k = e * T + f;
      b.comp[k] = adam_update(b.comp[k], b.g_comp[k], b.m_comp[k], b.v_comp[k], a);
    }
  }
  // torch.clamp semantics: NaN stays NaN (fmax/fmin would replace it)
  for (int f = 0; f < T; ++f) {
    const double c = b.comp[e * T + f];
    b.comp[e * T + f] = c < cfg.comp_min ? cfg.comp_min : c;
  }
  // group 2: targets, then clamp to the fingertip box
  if (cfg.lr[2] != 0.0) {
    a.step_size = -(cfg.lr[2] / bc1);
    for (int j = 0; j < 3 * T; ++j) {
      const int64_t k = e * 3 * T + j;
      b.target[k] = adam_update(b.target[k], b.g_target[k], b.m_target[k], b.v_target[k], a);
    }
  }
  if (cfg.clamp_target)
    for (int j = 0; j < 3 * T; ++j) {
      const int64_t k = e * 3 * T + j;
      double x = b.target[k];
      x = x < cfg.target_lb[j] ? cfg.target_lb[j] : x;
      b.target[k] = x > cfg.target_ub[j] ? cfg.target_ub[j] : x;
    }
  // groups 3, 4: palm position / orientation
  if (cfg.lr[3] != 0.0) {
    a.step_size = -(cfg.lr[3] / bc1);
    for (int i = 0; i < 3; ++i) {
      const int64_t k = 3 * e + i;
      b.palm_pos[k] = adam_update(b.palm_pos[k], b.g_palm_pos[k], b.m_palm_pos[k], b.v_palm_pos[k], a);
    }
  }
  if (cfg.lr[4] != 0.0) {
    a.step_size = -(cfg.lr[4] / bc1);
    for (int i = 0; i < 3; ++i) {
      const int64_t k = 3 * e + i;
      b.palm_ori[k] = adam_update(b.palm_ori[k], b.g_palm_ori[k], b.m_palm_ori[k], b.v_palm_ori[k], a);
    }
  }
}

}  // namespace

extern "C" int cdx_optimizer_step(const cdx_adam* cfg, const cdx_opt_buffers* buf, int64_t E, int32_t n_dofs,
                                  int32_t n_tips, int32_t iteration, cdx_stream_t stream) {
  if (!cfg || !buf || E < 0 || n_dofs < 0 || n_dofs > CDX_MAX_DOFS || n_tips <= 0 || n_tips > CDX_MAX_TIPS ||
      iteration < 0)
    return CDX_EINVAL;
  if (E == 0) return CDX_OK;
  const cdx_opt_buffers& b = *buf;
  if (!b.q || !b.comp || !b.target || !b.palm_pos || !b.palm_ori || !b.g_q || !b.g_comp || !b.g_target ||
      !b.g_palm_pos || !b.g_palm_ori || !b.m_q || !b.v_q || !b.m_comp || !b.v_comp || !b.m_target || !b.v_target ||
      !b.m_palm_pos || !b.v_palm_pos || !b.m_palm_ori || !b.v_palm_ori || !b.total_loss || !b.total_margin ||
      !b.opt_value || !b.opt_margin || !b.opt_q || !b.opt_comp || !b.opt_target || !b.opt_palm)
    return CDX_EINVAL;
  hipLaunchKernelGGL(optimizer_step_kernel, dim3((unsigned)((E + 63) / 64)), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), *cfg, *buf, E, n_dofs, n_tips, iteration);
  return hipGetLastError() == hipSuccess ? CDX_OK : CDX_ELAUNCH;
}
