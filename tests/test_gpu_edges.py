"""Edge cases of the HIP path against the oracle: empty and single-element
batches, inducing-point counts around the 64-row factor block and the 256-column GEMM tile,
a large GPIS (N = 4000), queries on / far from the training points.  GPU only."""
import numpy as np
import pytest
import torch

from tests._helpers import oracle_gpis_at, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _random_gpis(n, seed, kernel="tps"):
    """Sphere-surface points + a few inside/outside anchors, the in-repo fit recipe's structure."""
    from compliancedex_amd import GPIS
    from oracle.cdx_oracle import OracleGPIS
    rng = np.random.default_rng(seed)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    X1 = 0.05 * d
    y = np.zeros((n, 1))
    noise = np.full(n, 0.005)
    k = min(4, n)
    X1[:k] *= 3.0
    y[:k] = 0.1
    noise[:k] = 0.2
    g = GPIS(0.08, 1.0, kernel=kernel)
    g.fit(torch.from_numpy(X1).to(DEV), torch.from_numpy(y).to(DEV), noise=torch.from_numpy(noise).to(DEV))
    ref = OracleGPIS.fit(X1, y, noise, bias=1.0, kernel=kernel, sigma=0.08)
    return g, ref, X1


def _check_pred(g, ref, X, tm=1e-8, ts=1e-7):
    Xt = torch.from_numpy(X).to(DEV).requires_grad_(True)
    mean, std = g.pred(Xt)
    (mean.sum() + std.sum()).backward()
    r = oracle_gpis_at(ref, X, with_std=True)
    assert rel_err(mean.detach().cpu(), r["mean"]) < tm
    assert rel_err(std.detach().cpu(), r["std"]) < ts
    assert rel_err(Xt.grad.cpu(), r["gmean"] + r["gstd"]) < ts


@pytest.mark.parametrize("n", [1, 7, 63, 64, 65, 255, 256, 257, 513])
def test_gpis_ragged_inducing_counts(n):
    g, ref, X1 = _random_gpis(n, seed=n)
    rng = np.random.default_rng(100 + n)
    X = 0.08 * rng.standard_normal((300, 3))
    _check_pred(g, ref, X)


@pytest.mark.parametrize("kernel", ["rbf", "joint"])
def test_gpis_other_kernels_ragged(kernel):
    g, ref, X1 = _random_gpis(300, seed=3, kernel=kernel)
    X = 0.08 * np.random.default_rng(4).standard_normal((200, 3))
    _check_pred(g, ref, X, tm=1e-7, ts=1e-6)


def test_gpis_large_inducing_set():
    """N = 4000 (N_pad 4096, 16 column stripes: the XCD pairing's other branch), 1000 queries."""
    g, ref, X1 = _random_gpis(4000, seed=11)
    X = 0.08 * np.random.default_rng(12).standard_normal((1000, 3))
    idx = np.random.default_rng(13).choice(1000, 60, replace=False)
    Xt = torch.from_numpy(X).to(DEV).requires_grad_(True)
    mean, std = g.pred(Xt)
    std.sum().backward()
    r = oracle_gpis_at(ref, X[idx], with_std=True)
    assert rel_err(mean.detach().cpu().numpy()[idx], r["mean"]) < 1e-7
    assert rel_err(std.detach().cpu().numpy()[idx], r["std"]) < 1e-6
    assert rel_err(Xt.grad.cpu().numpy()[idx], r["gstd"]) < 1e-6


@pytest.mark.parametrize("n", [1800, 2000, 2047])
def test_gpis_whitened_column_shift_stripe_path(n):
    """≥ 4096 queries: one workgroup per (query tile, stripe), not split-K, with the whitened pass's
    padding columns shifted in front of stripe 0 (N_pad − N = 248 → 240, 48, 1 → 0)."""
    g, ref, X1 = _random_gpis(n, seed=20 + n)
    X = 0.08 * np.random.default_rng(21).standard_normal((4200, 3))
    idx = np.random.default_rng(22).choice(4200, 50, replace=False)
    Xt = torch.from_numpy(X).to(DEV).requires_grad_(True)
    mean, std = g.pred(Xt)
    std.sum().backward()
    r = oracle_gpis_at(ref, X[idx], with_std=True)
    assert rel_err(std.detach().cpu().numpy()[idx], r["std"]) < 1e-7
    assert rel_err(Xt.grad.cpu().numpy()[idx], r["gstd"]) < 1e-6


@pytest.mark.parametrize("m", [300, 16500])
def test_gpis_oversized_padding(monkeypatch, m):
    """A C-ABI state padded by ≥ 256 (N = 200, N_pad = 512): the whitened pass's column shift is
    capped below one stripe; split-K (300 queries) and stripe (16 500 queries) paths."""
    from compliancedex_amd import _native as N
    monkeypatch.setattr(N, "NPAD_ALIGN", 512)
    g, ref, X1 = _random_gpis(200, seed=31)
    assert g.native_state().desc.N_pad == 512
    X = 0.08 * np.random.default_rng(32).standard_normal((m, 3))
    idx = np.random.default_rng(33).choice(m, 50, replace=False)
    Xt = torch.from_numpy(X).to(DEV).requires_grad_(True)
    mean, std = g.pred(Xt)
    std.sum().backward()
    r = oracle_gpis_at(ref, X[idx], with_std=True)
    assert rel_err(std.detach().cpu().numpy()[idx], r["std"]) < 1e-7
    assert rel_err(Xt.grad.cpu().numpy()[idx], r["gstd"]) < 1e-6


def test_gpis_queries_on_and_far_from_training_points():
    g, ref, X1 = _random_gpis(500, seed=5)
    X = np.vstack([X1[:50], X1[50:100] + 1e-9, 5.0 * np.ones((3, 3)), -5.0 * np.ones((3, 3))])
    Xt = torch.from_numpy(X).to(DEV)
    mean, std = g.pred(Xt)
    r = oracle_gpis_at(ref, X, with_std=False)
    assert rel_err(mean.cpu(), r["mean"]) < 1e-8
    rs = ref.pred(torch.from_numpy(X))[1].numpy()
    # on a training point std ≈ its noise level (≪ k0): absolute agreement, relative to k0^½
    assert np.abs(std.cpu().numpy() - rs).max() < 1e-6 * np.sqrt(float(ref.R) ** 3)


def test_gpis_empty_and_single_query():
    g, ref, X1 = _random_gpis(100, seed=6)
    X0 = torch.zeros(0, 3, dtype=torch.float64, device=DEV, requires_grad=True)
    m0, s0 = g.pred(X0)
    assert m0.shape == (0,) and s0.shape == (0,)
    (m0.sum() + s0.sum()).backward()
    assert X0.grad.shape == (0, 3)
    assert g.compute_normal(torch.zeros(0, 3, dtype=torch.float64, device=DEV)).shape == (0, 3)
    _check_pred(g, ref, np.array([[0.01, -0.02, 0.03]]))


def _opt(hand, palm):
    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd.urdf import load_robot
    cfg = load_robot(hand)["config"]
    return ProbabilisticGraspOptimizer(hand, cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                       ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device=DEV), cfg


def test_closure_single_candidate_vs_oracle():
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs, stored_gpis
    from oracle.cdx_oracle import OracleChain, OracleGPIS, OracleProblem, closure_with_grads
    import os
    from tests._helpers import DATA
    opt, cfg = _opt("allegro", np.zeros((1, 6)))
    q, comp, target, palm = prob_inputs(cfg["ref_q"], 1, seed=2, spread=True)
    noise = np.random.default_rng(3).random((3, 3, 3))
    t = [torch.from_numpy(a).to(DEV).requires_grad_(True) for a in (q, comp, target, palm[:, :3], palm[:, 3:])]
    opt.closure(*t, 1, stored_gpis("banana", DEV), 1, kabsch_noise=torch.from_numpy(noise).to(DEV))
    prob = OracleProblem(OracleChain(load_robot("allegro")["bodies"]), cfg["ee_link_name"], cfg["ee_link_offset"],
                         cfg["ref_q"], OracleGPIS.from_npz(os.path.join(DATA, "gpis_states", "banana_state.npz")))
    ref = closure_with_grads(prob, q, comp, target, palm, noise)
    assert rel_err(opt.total_loss.cpu(), ref["total_loss"]) < 1e-4
    for k, x in zip(("grad_q", "grad_comp", "grad_target", "grad_palm_pos", "grad_palm_ori"), t):
        assert rel_err(x.grad.cpu(), ref[k]) < 1e-4, k


def test_closure_and_primitives_with_empty_batch():
    from compliancedex_amd import DifferentiableRobotModel, compute_sdf
    from compliancedex_amd.workloads import stored_gpis
    opt, cfg = _opt("allegro", np.zeros((0, 6)))
    f64 = dict(dtype=torch.float64, device=DEV)
    t = [torch.zeros(0, 16, **f64), torch.zeros(0, 4, **f64), torch.zeros(0, 4, 3, **f64), torch.zeros(0, 3, **f64),
         torch.zeros(0, 3, **f64)]
    loss = opt.closure(*t, 1, stored_gpis("banana", DEV), 0)
    assert float(loss) == 0.0 and opt.total_loss.shape == (0,)
    m = DifferentiableRobotModel("allegro", device=DEV)
    pos, quat = m.compute_forward_kinematics(torch.zeros(0, 16, device=DEV), cfg["ee_link_name"])
    assert pos.shape == (0, 12) and quat.shape == (0, 16)
    faces = torch.rand(5, 3, 3, device=DEV)
    d, s, n, c = compute_sdf(torch.zeros(0, 3, device=DEV), faces)
    assert d.shape == (0,) and c.shape == (0, 3)
    d, s, n, c = compute_sdf(torch.rand(7, 3, device=DEV), faces[:1])  # a single face
    assert torch.isfinite(d).all() and set(s.cpu().tolist()) <= {-1, 1}
