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


def oracle_gpis(state):
    from oracle.cdx_oracle import OracleGPIS
    if state == "synthetic2000":
        d = golden("gpis_synthetic2000.npz")
        return OracleGPIS.fit(d["syn_X1"], d["syn_y"], d["syn_noise"], bias=1.0)
    return OracleGPIS.from_npz(os.path.join(DATA, "gpis_states", f"{state}_state.npz"))


def oracle_chain(robot):
    from compliancedex_amd.urdf import load_robot
    from oracle.cdx_oracle import OracleChain
    c = load_robot(robot)
    return OracleChain(c["bodies"]), c


def oracle_problem(hand, state):
    from oracle.cdx_oracle import OracleProblem
    chain, c = oracle_chain(hand)
    cfg = c["config"]
    return OracleProblem(chain, cfg["ee_link_name"], cfg["ee_link_offset"], cfg["ref_q"], oracle_gpis(state))


def rel_err(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def product_chain(robot):
    from compliancedex_amd.chain import Chain
    from compliancedex_amd.urdf import load_robot
    return Chain(load_robot(robot))


def host_problem(hand):
    from compliancedex_amd.problem import build_problem
    ch = product_chain(hand)
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
