"""Config-4 TorchSDF forward as a profiling child: 3 × 65 536 random points around the 16 384-face banana
(the c4 case's points), the three cdx_sdf_forward calls of one SDF/Kin iteration, repeated REPS times.

  python tools/sdf_child.py [REPS]        (under rocprofv3 --pmc / --kernel-trace; tools/pmc_sdf.sh)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from compliancedex_amd.torchsdf import compute_sdf  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(reps):
    dev = "cuda"
    torch.manual_seed(0)
    faces = torch.from_numpy(np.load(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_faces.npy"))).to(dev)
    lo, hi = faces.reshape(-1, 3).min(0)[0], faces.reshape(-1, 3).max(0)[0]
    pts = [lo - 0.02 + (hi - lo + 0.04) * torch.rand(65536, 3, device=dev) for _ in range(3)]
    deflated = faces * 0.9
    with torch.no_grad():
        for _ in range(reps):
            for i, f in enumerate((deflated, faces, faces)):
                compute_sdf(pts[i], f)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
