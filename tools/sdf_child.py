"""Config-4 TorchSDF forward as a profiling child: the three queries of one SDF/Kin iteration (4E fingertips vs
the deflated and the true 16 384-face banana, 4E targets vs the true mesh; E = 16 384, workloads.config4_kin_inputs)
on prepared meshes, repeated REPS times.

  python tools/sdf_child.py [REPS]        (under rocprofv3 --pmc / --kernel-trace; tools/pmc_sdf.sh)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps):
    from compliancedex_amd import DifferentiableRobotModel, PreparedMesh
    from compliancedex_amd.optimizers import _face_vertices
    from compliancedex_amd.workloads import banana_mesh, config4_kin_inputs
    dev = "cuda"
    links, offs, palm, q, target, comp = config4_kin_inputs(16384, device=dev)
    tips = (DifferentiableRobotModel("iiwa7_allegro", device=dev).compute_forward_kinematics(
        torch.from_numpy(q).to(dev), links, offsets=offs)[0].view(-1, 3) + torch.from_numpy(palm).to(dev)).contiguous()
    tg = torch.from_numpy(target).to(dev).view(-1, 3).contiguous()
    m = banana_mesh()
    faces = _face_vertices(m, dev)
    m.scale(0.9, center=[0, 0, 0])
    full, deflated = PreparedMesh(faces), PreparedMesh(_face_vertices(m, dev))
    from compliancedex_amd.torchsdf import QueryWorkspace
    ws_t, ws_g = QueryWorkspace(), QueryWorkspace()
    with torch.no_grad():
        for _ in range(reps):
            deflated.query(tips, workspace=ws_t)
            full.query(tips, workspace=ws_t, reuse_order=True)
            full.query(tg, workspace=ws_g)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
