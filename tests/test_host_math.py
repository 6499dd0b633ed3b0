"""The per-candidate device code (FK, Kabsch/SVD, cost, backward), compiled for the host,
checked against the reference's golden vectors and the oracle.  CPU only."""
import numpy as np
import pytest

from tests import _host
from tests._helpers import (golden, golden_names, host_problem, oracle_gpis, oracle_gpis_at, product_chain,
                            rel_err)

FK_CASES = golden_names("fk_")
CLOSURE_CASES = golden_names("closure_")


@pytest.mark.parametrize("name", FK_CASES)
def test_fk_host_vs_reference(name):
    d = golden(name)
    robot = "iiwa7_allegro" if name.startswith("fk_iiwa7") else name.split("_")[1]
    ch = product_chain(robot)
    desc = ch.descriptor([str(s) for s in d["links"]], d["offsets"].tolist())
    pos, quat = _host.fk_forward(desc, d["q"])
    assert rel_err(pos, d["pos"]) < 2e-6
    assert rel_err(quat, d["quat"]) < 2e-6
    gq = _host.fk_backward(desc, d["q"], d["cot"])
    assert rel_err(gq, d["grad_q"]) < 2e-5


def test_svd3_accuracy():
    rng = np.random.default_rng(0)
    for trial in range(200):
        if trial % 2:
            a, b = rng.standard_normal(3), rng.standard_normal(3)
            H = np.outer(a, b) * 10 + 1e-6 * rng.random((3, 3))  # rank-1 + noise, as at init
        else:
            H = rng.standard_normal((3, 3))
        U, S, V = _host.svd3(H)
        assert np.all(np.diff(S) <= 0)
        assert np.abs(U @ np.diag(S) @ V.T - H).max() < 1e-14 * np.abs(H).max() * 10
        assert np.abs(U.T @ U - np.eye(3)).max() < 1e-12
        assert np.abs(V.T @ V - np.eye(3)).max() < 1e-12
        S_ref = np.linalg.svd(H, compute_uv=False)
        assert np.abs(S - S_ref).max() < 1e-14 * S_ref[0] * 10


@pytest.mark.parametrize("name", CLOSURE_CASES)
def test_closure_host_vs_reference(name):
    d = golden(name)
    prob = host_problem(str(d["hand"]), d)
    X = _host.closure_queries(prob, d["q"], d["target"], d["palm"])
    E, T = d["q"].shape[0], prob.chain.n_tips
    pre = X[(prob.n_query_levels + 1) * E * T:(prob.n_query_levels + 2) * E * T].reshape(E, T, 3)
    assert rel_err(pre, d["pregrasp_tip"]) < 1e-6  # float32 FK, op order differs from torch
    g = oracle_gpis(str(d["state"]))
    Ms = prob.n_query_levels * E * T
    gp = oracle_gpis_at(g, X, with_std=False)
    gs = oracle_gpis_at(g, X[:Ms], with_std=True)
    gp["std"], gp["gstd"] = gs["std"], gs["gstd"]
    out = _host.closure_cost(prob, d["q"], d["comp"], d["target"], d["palm"], d["noise"][0], gp)
    errs = {k: rel_err(out[k], d[k]) for k in ("total_loss", "total_margin", "grad_q", "grad_comp", "grad_target",
                                               "grad_palm_pos", "grad_palm_ori")}
    print(name, errs)
    assert all(v < 1e-4 for v in errs.values()), errs


@pytest.mark.parametrize("name", golden_names("collision_"))
def test_collision_host_vs_reference(name):
    """compute_collision_loss (:671-701): pair / anchor-floor / palm-floor terms and gradients."""
    from tests._helpers import collision_desc
    d = golden(name)
    cost, g_q, g_palm = _host.collision(collision_desc(str(d["hand"])), d["q"], d["palm"])
    # masks bit-exact; floats at the north-star 1e-4 bar: the anchors come from f32 FK and 1/z,
    # 1/d amplify its last-ulp differences near the floor (measured ≤ 1.2e-5 on these fixtures)
    assert np.array_equal(cost != 0, d["cost"] != 0)
    assert rel_err(cost, d["cost"]) < 1e-4
    assert rel_err(g_q, d["grad_q"]) < 1e-4
    assert rel_err(g_palm, d["grad_palm"]) < 1e-4


@pytest.mark.parametrize("name", golden_names("force_eq_"))
def test_force_eq_host_vs_reference(name):
    """force_eq_reward (:73-118): the ForceEq code shared by the closure and the standalone op."""
    from compliancedex_amd.force_eq import force_eq_descriptor
    d = golden(name)
    desc = force_eq_descriptor(4, float(d["mu"]) if float(d["mu"]) != 1 else 1, float(d["mass"]),
                               10.0 if bool(d["gravity"]) else None, COM=d["com"].tolist())
    out = _host.force_eq(desc, d["tip"], d["target"], d["comp"], d["normal"], d["noise"], d["cr"], d["cf"])
    for k in ("reward", "margin", "force_norm"):
        assert rel_err(out[k], d[k]) < 1e-9, k
    for k in ("grad_tip", "grad_target", "grad_comp"):
        assert rel_err(out[k], d[k]) < 1e-6, (k, rel_err(out[k], d[k]))
