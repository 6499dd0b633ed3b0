"""Pins the oracle (oracle/cdx_oracle.py) against vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from tests._helpers import golden, golden_names, oracle_chain, oracle_gpis, oracle_problem, rel_err

GPIS_CASES = [n[len("gpis_"):-4] for n in golden_names("gpis_")]
FK_CASES = golden_names("fk_")
CLOSURE_CASES = golden_names("closure_")
NORMAL_CASES = golden_names("normals_")


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
    prob = oracle_problem(str(d["hand"]), str(d["state"]), d)
    out = closure_with_grads(prob, d["q"], d["comp"], d["target"], d["palm"], d["noise"][0])
    assert rel_err(out["pregrasp_tip"], d["pregrasp_tip"]) < 1e-9
    assert rel_err(out["total_loss"], d["total_loss"]) < 1e-8
    assert rel_err(out["total_margin"], d["total_margin"]) < 1e-8
    for k in ("grad_q", "grad_comp", "grad_target", "grad_palm_pos", "grad_palm_ori"):
        assert rel_err(out[k], d[k]) < 1e-6, k


@pytest.mark.parametrize("name", [n for n in CLOSURE_CASES if n.startswith("closure_iiwa7")])
def test_collision_iiwa7(name):
    """compute_collision_loss on the 23-DOF chain, fingertip anchors, all six pairs (:671-701)."""
    from oracle.cdx_oracle import collision_loss
    d = golden(name)
    chain, _ = oracle_chain("iiwa7_allegro")
    q = torch.from_numpy(d["q"]).requires_grad_(True)
    palm = torch.from_numpy(d["palm"]).requires_grad_(True)
    cost = collision_loss(chain, [str(s) for s in d["links"]], d["offsets"].tolist(), d["pairs"], q, palm)
    cost.sum().backward()
    assert rel_err(cost.detach(), d["coll_cost"]) < 1e-12
    assert rel_err(q.grad, d["coll_grad_q"]) < 1e-6  # f32 FK backward: 6e-8 measured
    assert rel_err(palm.grad, d["coll_grad_palm"]) < 1e-12


@pytest.mark.parametrize("name", golden_names("collision_"))
def test_collision(name):
    from oracle.cdx_oracle import collision_loss
    d = golden(name)
    hand = str(d["hand"])
    chain, c = oracle_chain(hand)
    cfg = c["config"]
    q = torch.from_numpy(d["q"]).requires_grad_(True)
    palm = torch.from_numpy(d["palm"]).requires_grad_(True)
    cost = collision_loss(chain, cfg["collision_links"], cfg["collision_offsets"], cfg["collision_pairs"], q, palm)
    cost.sum().backward()
    assert rel_err(cost.detach(), d["cost"]) < 1e-12
    assert rel_err(q.grad, d["grad_q"]) < 1e-6
    assert rel_err(palm.grad, d["grad_palm"]) < 1e-12


@pytest.mark.parametrize("name", NORMAL_CASES)
def test_normals_index_and_multinormals(name):
    """compute_normal(X, index) and compute_multinormals (gpis.py:63-111)."""
    d = golden(name)
    g = oracle_gpis(name[len("normals_"):-4])
    X = torch.from_numpy(d["X"])
    for i in range(3):
        nrm, w = g.compute_normal(X, d[f"index{i}"].tolist())
        assert rel_err(nrm, d[f"normal_index{i}"]) < 1e-12
        assert abs(float(w) - float(d[f"weight_index{i}"])) <= 1e-9 * abs(float(d[f"weight_index{i}"]))
    for S in (3, 5):
        for dim in (2, 3):
            Xd = X if dim == 2 else X.view(-1, 4, 3)
            nrms, ws = g.compute_multinormals(Xd, S)
            assert nrms.shape == d[f"multi{S}_{dim}d_normals"].shape
            assert rel_err(nrms, d[f"multi{S}_{dim}d_normals"]) < 1e-12
            assert rel_err(ws, d[f"multi{S}_{dim}d_weights"]) < 1e-9


@pytest.mark.parametrize("exp", ["lego", "realsense"])
def test_reference_results_are_allegro_fk(exp):
    """The reference's own saved outputs: contact = forward_kinematics(joint_angle, wrist) with the
    Allegro config offsets (optimize_pregrasp.py:1009, :1016-1020).  The files were written by the
    reference on a CUDA device: f32 FK rounding, 1.0e-7 relative measured → 1e-6."""
    d = golden(f"results_{exp}.npz")
    prob = oracle_problem("allegro", "banana")
    out = prob.forward_kinematics(torch.from_numpy(d["joint_angle"]), torch.from_numpy(d["wrist"]))
    assert rel_err(out.detach(), d["contact"]) < 1e-6


def test_kin_sdf_loop_oracle_vs_reference_run():
    """The oracle's Kin-mode loop (oracle.kin_sdf_loop: FK → 3 TorchSDF calls through the C oracle →
    force_eq_reward → costs → Adam, float32) against the reference's own KinGraspOptimizer run
    (golden mode_kin: 12 iterations, E = 1, replayed Kabsch noise; its TorchSDF was the same C
    oracle, the reference's _C being absent).  This pins the oracle the config-4 GPU test compares
    the full-size SDF loop with."""
    import os
    from compliancedex_amd.optimizers import TriangleMesh, _face_vertices
    from oracle.cdx_oracle import kin_sdf_loop
    from tests._sdf_oracle import oracle_sdf
    from tests.conftest import REPO
    d = golden("mode_kin.npz")
    chain, robot = oracle_chain("allegro")
    cfg = robot["config"]
    mesh = TriangleMesh.from_npz(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_mesh.npz"))
    faces = _face_vertices(mesh, "cpu")
    faces_def = _face_vertices(mesh.scale(0.9, center=[0, 0, 0]), "cpu")
    loss, oq, oc, ot, flag = kin_sdf_loop(chain, cfg["ee_link_name"], cfg["ee_link_offset"], d["palm3"], cfg["ref_q"],
                                          d["q"], d["target"], d["comp"], 1, faces, faces_def, oracle_sdf,
                                          d["noise"], int(d["iters"]))
    trace = loss.sum(dim=1).double().numpy()
    assert np.abs(trace - d["loss_trace"]).max() <= 1e-5 * np.abs(d["loss_trace"]).max(), (trace, d["loss_trace"])
    # float32 end to end (as the reference): 12 Adam steps of f32 FK / Kabsch rounding → measured 1.9e-5
    for i, x in enumerate((oq, oc, ot)):
        assert rel_err(x.double(), d[f"out{i}"]) < 1e-4, i
    assert flag == bool(d["flag"])


def test_kin_sdf_loop_resumes_from_adam_state():
    """oracle.kin_sdf_loop resumed from a loop state (parameters, Adam's moments and step count — the form
    test_config4_kin_divergence_vs_oracle injects from the GPU's loop) continues the uninterrupted run bit for bit:
    12 iterations of the reference's mode_kin case straight, against 5 + 7 with the state handed over."""
    import os
    from compliancedex_amd.optimizers import TriangleMesh, _face_vertices
    from oracle.cdx_oracle import kin_sdf_loop
    from tests._sdf_oracle import oracle_sdf
    from tests.conftest import REPO
    d = golden("mode_kin.npz")
    chain, robot = oracle_chain("allegro")
    cfg = robot["config"]
    mesh = TriangleMesh.from_npz(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_mesh.npz"))
    faces = _face_vertices(mesh, "cpu")
    faces_def = _face_vertices(mesh.scale(0.9, center=[0, 0, 0]), "cpu")
    args = (chain, cfg["ee_link_name"], cfg["ee_link_offset"], d["palm3"], cfg["ref_q"])
    iters, k = int(d["iters"]), 5
    full, *_ = kin_sdf_loop(*args, d["q"], d["target"], d["comp"], 1, faces, faces_def, oracle_sdf, d["noise"], iters)
    st = {}
    head, *_ = kin_sdf_loop(*args, d["q"], d["target"], d["comp"], 1, faces, faces_def, oracle_sdf, d["noise"][:k], k,
                            state_out=st)
    tail, *_ = kin_sdf_loop(*args, st["q"], st["target"], st["comp"], 1, faces, faces_def, oracle_sdf, d["noise"][k:],
                            iters - k, adam_state=st["adam_state"])
    assert torch.equal(torch.cat([head, tail]), full)


def test_oracle_kabsch_nonfinite_rows():
    """The oracle's Kabsch factors only the finite rows (the reference's CUDA SVD returns NaN for a diverged row, where
    torch's CPU LAPACK raises): the finite rows equal the all-finite call's, a NaN row's rotation is NaN."""
    from oracle.cdx_oracle import kabsch
    rng = np.random.default_rng(3)
    S1, S2 = torch.from_numpy(rng.standard_normal((6, 5, 3))), torch.from_numpy(rng.standard_normal((6, 5, 3)))
    w, noise = torch.from_numpy(rng.random((6, 5))), torch.from_numpy(rng.random((6, 3, 3)))
    R, t, flip = kabsch(S1, S2, w, noise)
    S1b = S1.clone()
    S1b[2, 1, 0] = float("nan")
    Rb, tb, _ = kabsch(S1b, S2, w, noise)
    keep = torch.tensor([0, 1, 3, 4, 5])
    assert torch.equal(Rb[keep], R[keep]) and torch.equal(tb[keep], t[keep])
    assert torch.isnan(Rb[2]).all()


def test_sdf_mode_loop_oracle_vs_reference_run():
    """The oracle's SDF-mode loop (oracle.sdf_mode_loop: 3 TorchSDF calls through the C oracle → force_eq_reward
    → costs → RMSprop → box clamps, float32) against the reference's own SDFGraspOptimizer run (golden mode_sdf:
    12 iterations, E = 1, replayed Kabsch noise, its TorchSDF the same C oracle).  This pins the oracle the
    fused SDF-mode GPU test at E = 16 384 compares with."""
    import os
    from compliancedex_amd.optimizer import FINGERTIP_LB, FINGERTIP_UB
    from compliancedex_amd.optimizers import TriangleMesh, _face_vertices
    from oracle.cdx_oracle import sdf_mode_loop
    from tests._sdf_oracle import oracle_sdf
    from tests.conftest import REPO
    d = golden("mode_sdf.npz")
    mesh = TriangleMesh.from_npz(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_mesh.npz"))
    faces = _face_vertices(mesh, "cpu")
    faces_def = _face_vertices(mesh.scale(0.9, center=[0, 0, 0]), "cpu")
    loss, ot, oc, og, flag = sdf_mode_loop(d["tips"], d["target"], d["comp"], 1, faces, faces_def, oracle_sdf,
                                           d["noise"], int(d["iters"]), FINGERTIP_LB, FINGERTIP_UB)
    trace = loss.sum(dim=1).double().numpy()
    assert np.abs(trace - d["loss_trace"]).max() <= 1e-5 * np.abs(d["loss_trace"]).max(), (trace, d["loss_trace"])
    for i, x in enumerate((ot, oc, og)):
        assert rel_err(x.double(), d[f"out{i}"]) < 1e-5, i
    assert flag == bool(d["flag"])
