"""CPU study: does the reference's float32 Kin loop (oracle.kin_sdf_loop, pinned to the reference's mode_kin run)
go non-finite on config 4's inputs (workloads.config4_kin_inputs: iiwa7_allegro, banana mesh)?  Runs the oracle on
candidate slices for ITERS iterations with a random Kabsch noise tape and prints, per iteration, the count of
candidates whose loss is non-finite, and the first iteration of each diverged candidate.

  python tools/c4_divergence_cpu.py [n_candidates] [iters] [start] [comma-separated candidate list]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from compliancedex_amd.optimizers import TriangleMesh, _face_vertices  # noqa: E402
from compliancedex_amd.urdf import load_robot  # noqa: E402
from compliancedex_amd.workloads import CONFIG4_OFFSETS  # noqa: E402
from oracle.cdx_oracle import OracleChain, kin_sdf_loop  # noqa: E402
from tests import _sdf_oracle  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def inputs(E, seed=44, q_scale=0.05):
    """config4_kin_inputs with the fingertip centre from the oracle chain (no GPU here)."""
    c = load_robot("iiwa7_allegro")
    chain = OracleChain(c["bodies"])
    links = c["config"]["ee_link_name"]
    center = np.load(os.path.join(REPO, "compliancedex_amd", "data", "banana_center.npy"))
    tips0 = chain.forward_kinematics(torch.zeros(1, 23), links, CONFIG4_OFFSETS)[0].view(4, 3).double().mean(0).numpy()
    rng = np.random.default_rng(seed)
    q = (q_scale * rng.standard_normal((E, 23))).astype(np.float32)
    target = (np.tile(center, (E, 4, 1)) + 0.01 * rng.standard_normal((E, 4, 3))).astype(np.float32)
    comp = np.tile(np.array([10.0, 10.0, 10.0, 20.0], np.float32), (E, 1))
    return chain, links, (center - tips0).astype(np.float32), q, target, comp


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    start = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    torch.set_num_threads(8)
    E = 16384
    chain, links, palm, q, target, comp = inputs(E)
    sl = np.arange(start, start + n) if len(sys.argv) <= 4 else np.array([int(v) for v in sys.argv[4].split(',')])
    n = len(sl)
    mesh = TriangleMesh.from_npz(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_mesh.npz"))
    faces = _face_vertices(mesh, "cpu")
    faces_def = _face_vertices(mesh.scale(0.9, center=[0, 0, 0]), "cpu")
    # the GPU tool's tape (tools/c4_divergence_gpu.py): the same draw for all E candidates, sliced
    noise = np.random.default_rng(7).random((iters, E, 3, 3), dtype=np.float32)[:, sl]
    loss, oq, oc, ot, _ = kin_sdf_loop(chain, links, CONFIG4_OFFSETS, palm, [0.0] * 23, q[sl], target[sl], comp[sl], 1,
                                       faces, faces_def, _sdf_oracle.oracle_sdf, noise, iters)
    L = loss.numpy()
    bad = ~np.isfinite(L)
    first = np.where(bad.any(0), bad.argmax(0), -1)
    np.save(f"/tmp/c4_oracle_loss_{iters}_{start}_{n}.npy", L)
    print(json.dumps({"n": n, "iters": iters, "start": start,
                      "nonfinite_by_iter": [int(b) for b in bad.sum(1)],
                      "diverged": {int(sl[i]): int(first[i]) for i in range(n) if first[i] >= 0}}))


if __name__ == "__main__":
    main()
