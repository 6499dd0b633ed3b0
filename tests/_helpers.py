"""Shared test helpers: fixture loading and oracle construction from packaged data."""
import glob
import os

import numpy as np

from tests.conftest import GOLDEN, REPO

DATA = os.path.join(REPO, "compliancedex_amd", "data")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def golden_names(prefix):
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


FITTED_STATES = ("synthetic2000", "box")  # no stored state: refit from the fixture's X1/y/noise


def oracle_gpis(state):
    from oracle.cdx_oracle import OracleGPIS
    if state in FITTED_STATES:
        d = golden(f"gpis_{state}.npz")
        return OracleGPIS.fit(d["syn_X1"], d["syn_y"], d["syn_noise"], bias=1.0)
    return OracleGPIS.from_npz(os.path.join(DATA, "gpis_states", f"{state}_state.npz"))


def oracle_chain(robot):
    from compliancedex_amd.urdf import load_robot
    from oracle.cdx_oracle import OracleChain
    c = load_robot(robot)
    return OracleChain(c["bodies"]), c


def oracle_problem(hand, state, d=None):
    """OracleProblem for a hand's packaged config, or for a closure fixture ``d`` that carries its
    own fingertip links / offsets (the iiwa7_allegro cases: ref_q = 0)."""
    from oracle.cdx_oracle import OracleProblem
    chain, c = oracle_chain(hand)
    if d is not None and "links" in d.files:
        return OracleProblem(chain, [str(s) for s in d["links"]], d["offsets"].tolist(), [0.0] * chain.n_dofs,
                             oracle_gpis(state))
    cfg = c["config"]
    return OracleProblem(chain, cfg["ee_link_name"], cfg["ee_link_offset"], cfg["ref_q"], oracle_gpis(state))


def rel_err(a, b):
    """max|a − b| / max|b|.  NaNs must sit at the same positions in both (the reference's
    unclamped contact-margin log, optimize_pregrasp.py:708); they are then left out."""
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return float("inf")
    if na.all():
        return 0.0
    a, b = a[~na], b[~nb]
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def product_chain(robot):
    from compliancedex_amd.chain import Chain
    from compliancedex_amd.urdf import load_robot
    return Chain(load_robot(robot))


def host_problem(hand, d=None):
    """cdx_problem for a hand's packaged config, or for a closure fixture that carries its own
    fingertip links / offsets (iiwa7_allegro: ref_q = 0)."""
    from compliancedex_amd.problem import build_problem
    ch = product_chain(hand)
    if d is not None and "links" in d.files:
        return build_problem(ch.descriptor([str(s) for s in d["links"]], d["offsets"].tolist()), None,
                             ref_q=[0.0] * ch.n_dofs)
    cfg = ch.config
    return build_problem(ch.descriptor(cfg["ee_link_name"], cfg["ee_link_offset"]), None, ref_q=cfg["ref_q"])


def oracle_gpis_at(g, X, with_std):
    """mean/∇mean/normal (and std/∇std) at each row of X via the oracle's autograd."""
    import torch
    Xt = torch.from_numpy(np.ascontiguousarray(X)).requires_grad_(True)
    mean, std = g.pred(Xt)
    gmean, = torch.autograd.grad(mean.sum(), Xt, retain_graph=True)
    out = dict(mean=mean.detach().numpy(), gmean=gmean.numpy(),
               normal=g.compute_normal(torch.from_numpy(np.ascontiguousarray(X))).numpy())
    if with_std:
        gstd, = torch.autograd.grad(std.sum(), Xt)
        out.update(std=std.detach().numpy(), gstd=gstd.numpy())
    return out


def collision_desc(hand):
    """cdx_collision for a packaged hand's collision links / pairs (robot config), palm term on."""
    from compliancedex_amd.problem import build_collision
    ch = product_chain(hand)
    cfg = ch.config
    return build_collision(ch.descriptor(cfg["collision_links"], cfg["collision_offsets"]), cfg["collision_pairs"])


def assert_rel(a, b, tol, tag):
    """rel_err(a, b) < tol, and the measured error logged as a JSON line to $CDX_PARITY_LOG
    (tools/parity_report.py collects them: the tolerances are set ~10× the measured values)."""
    import json
    import os
    err = rel_err(a, b)
    path = os.environ.get("CDX_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0]
            f.write(json.dumps({"test": test, "tag": tag, "err": err, "tol": tol}) + "\n")
    assert err < tol, (tag, err, tol)
    return err
