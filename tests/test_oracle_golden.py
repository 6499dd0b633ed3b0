"""Pins the oracle (oracle/cdx_oracle.py) against vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from tests._helpers import golden, golden_names, oracle_chain, oracle_gpis, oracle_problem, rel_err

GPIS_CASES = [n[len("gpis_"):-4] for n in golden_names("gpis_")]
FK_CASES = golden_names("fk_")
CLOSURE_CASES = golden_names("closure_")


@pytest.mark.parametrize("state", GPIS_CASES)
def test_gpis_pred_normal(state):
    d = golden(f"gpis_{state}.npz")
    g = oracle_gpis(state)
    X = torch.from_numpy(d["X"]).requires_grad_(True)
    mean, std = g.pred(X)
    ((mean * torch.from_numpy(d["cm"])).sum() + (std * torch.from_numpy(d["cs"])).sum()).backward()
    tol = 1e-9 if state != "synthetic2000" else 1e-6
    assert rel_err(mean.detach(), d["mean"]) < tol
    assert rel_err(std.detach(), d["std"]) < tol
    assert rel_err(X.grad, d["grad_X"]) < tol
    assert rel_err(g.compute_normal(torch.from_numpy(d["X"])), d["normal"]) < tol
    m3, s3 = g.pred(torch.from_numpy(d["X"]).view(-1, 4, 3))
    assert m3.shape == d["mean3"].shape
    assert rel_err(m3, d["mean3"]) < tol and rel_err(s3, d["std3"]) < tol


@pytest.mark.parametrize("name", FK_CASES)
def test_fk(name):
    d = golden(name)
    robot = name.split("_")[1] if not name.startswith("fk_iiwa7") else "iiwa7_allegro"
    chain, _ = oracle_chain(robot)
    q = torch.from_numpy(d["q"]).requires_grad_(True)
    pos, quat = chain.forward_kinematics(q, [str(s) for s in d["links"]], d["offsets"].tolist())
    (pos * torch.from_numpy(d["cot"])).sum().backward()
    assert rel_err(pos.detach(), d["pos"]) < 1e-5
    assert rel_err(quat.detach(), d["quat"]) < 1e-5
    assert rel_err(q.grad, d["grad_q"]) < 1e-4


@pytest.mark.parametrize("name", CLOSURE_CASES)
def test_closure(name):
    from oracle.cdx_oracle import closure_with_grads
    d = golden(name)
    prob = oracle_problem(str(d["hand"]), str(d["state"]))
    out = closure_with_grads(prob, d["q"], d["comp"], d["target"], d["palm"], d["noise"][0])
    assert rel_err(out["pregrasp_tip"], d["pregrasp_tip"]) < 1e-9
    assert rel_err(out["total_loss"], d["total_loss"]) < 1e-8
    assert rel_err(out["total_margin"], d["total_margin"]) < 1e-8
    for k in ("grad_q", "grad_comp", "grad_target", "grad_palm_pos", "grad_palm_ori"):
        assert rel_err(out[k], d[k]) < 1e-6, k
