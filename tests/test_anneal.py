"""Annealing outer loop (config 5, build-defined: the reference's simanneal.py is empty).
CPU: the Metropolis / best-state bookkeeping against a scripted inner optimiser.  GPU: the loop
over the real fused inner optimisation."""
import numpy as np
import pytest
import torch

from compliancedex_amd.anneal import PregraspAnnealer


class _Scripted:
    """Duck-typed inner optimiser: returns the proposal shifted by +1 and a scripted best loss."""
    num_iters = 30

    def __init__(self, losses):
        self.losses = list(losses)
        self.calls = []

    def optimize(self, q, target, comp, mu, gpis, verbose=False, init_palm=None):
        self.calls.append(q.clone())
        self.best_loss = self.losses.pop(0)
        E, T = comp.shape
        return q + 1, comp, target, init_palm, torch.ones(E, T, dtype=torch.float64)


def test_metropolis_and_best_tracking():
    E = 4
    inf = float("inf")
    losses = [torch.tensor([5.0, 5.0, float("nan"), 1.0], dtype=torch.float64),
              torch.tensor([4.0, 500.0, 3.0, 2.0], dtype=torch.float64),
              torch.tensor([6.0, 6.0, 2.0, 0.5], dtype=torch.float64)]
    opt = _Scripted(losses)
    a = PregraspAnnealer(opt, None, temperature=1e-9, cooling=1.0, q_sigma=0.0, palm_pos_sigma=0.0,
                         palm_ori_sigma=0.0)
    q = torch.zeros(E, 2, dtype=torch.float64)
    best = a.run(q, torch.zeros(E, 4, 3, dtype=torch.float64), torch.ones(E, 4, dtype=torch.float64),
                 torch.zeros(E, 6, dtype=torch.float64), outer_steps=3)
    # step 0 accepts every finite loss (Δ = −inf); NaN is rejected
    # step 1: candidate 0 improves (accept), 1 worsens at T→0 (reject), 2 first finite (accept), 3 worsens (reject)
    # step 2: 0 worsens, 1 improves vs its current 5 (6 > 5: reject), 2 improves, 3 improves
    assert best["loss"].tolist() == [4.0, 5.0, 2.0, 0.5]
    assert best["accepted"].tolist() == [2, 1, 2, 2]
    # proposals start from the accepted state: candidate 0 accepted twice → q advanced twice
    assert opt.calls[2][:, 0].tolist() == [2.0, 1.0, 1.0, 1.0]
    assert best["q"][:, 0].tolist() == [2.0, 1.0, 2.0, 2.0]
    assert not torch.isinf(best["loss"]).any() and inf not in best["loss"].tolist()


def test_requires_best_iterate_window():
    class Short(_Scripted):
        num_iters = 20
    with pytest.raises(ValueError, match="num_iters"):
        PregraspAnnealer(Short([]), None)


@pytest.mark.gpu
def test_anneal_on_device_improves_and_is_deterministic():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs, stored_gpis
    dev = torch.device("cuda")
    cfg = load_robot("allegro")["config"]
    E = 64
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=3, spread=True)
    g = stored_gpis("banana", dev)
    t = [torch.from_numpy(x).to(dev) for x in (q, target, comp, palm)]

    def run(seed):
        opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                          ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device=dev,
                                          num_iters=30, seed=7)
        return PregraspAnnealer(opt, g, seed=seed).run(*t, outer_steps=3)

    b1, b2 = run(1), run(1)
    for k in ("loss", "q", "palm", "margin"):
        assert torch.equal(b1[k], b2[k]), k
    fin = torch.isfinite(b1["loss"])
    assert fin.sum() > E // 2
    # a single inner optimisation from the same start is never better than the annealed best
    opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                      ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device=dev,
                                      num_iters=30, seed=7)
    opt.optimize(t[0], t[1], t[2], 1, g, verbose=False)
    one = opt.best_loss
    assert torch.all(b1["loss"][fin] <= one[fin] + 1e-9)
