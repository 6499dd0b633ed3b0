"""Config 4's fused Kin loop (workloads.config4_kin_inputs, E = 16 384, iiwa7_allegro, banana mesh) for ITERS iterations
with a recorded Kabsch noise tape (numpy default_rng(TAPE_SEED).random((iters, E, 3, 3)) in float32, the same tape
tools/c4_divergence_cpu.py and the oracle comparison regenerate), per-candidate losses traced.  Writes
gpurun_out/c4_div_<iters>.npz (loss rows [iters, E] f64, best q / comp / target) and prints the count of candidates
whose loss is non-finite per iteration and the first such iteration of each.

  python tools/c4_divergence_gpu.py [iters]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TAPE_SEED = 7


def main():
    from compliancedex_amd import KinGraspOptimizer
    from compliancedex_amd.workloads import banana_mesh, config4_kin_inputs
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    dev = torch.device("cuda:0")
    E = 16384
    links, offs, palm, q, target, comp = config4_kin_inputs(E, device=dev)
    tape = np.random.default_rng(TAPE_SEED).random((iters, E, 3, 3), dtype=np.float32)
    noise = [torch.from_numpy(tape[s]).to(dev) for s in range(iters)]
    kin = KinGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=palm.tolist(), num_iters=iters,
                            optimize_target=True, ref_q=[0.0] * 23, device=dev)
    x = [torch.from_numpy(a).to(dev) for a in (q, target, comp)]
    res = kin.optimize(*x, 1, banana_mesh(), verbose=False, kabsch_noise=noise, trace_rows=True, fused=True)
    torch.cuda.synchronize()
    L = torch.stack(kin.loss_rows).cpu().numpy()
    bad = ~np.isfinite(L)
    first = np.where(bad.any(0), bad.argmax(0), -1)
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/c4_div_{iters}.npz", loss=L, first=first,
                        q=res[0].detach().cpu().numpy(), comp=res[1].detach().cpu().numpy(),
                        target=res[2].detach().cpu().numpy())
    div = np.nonzero(first >= 0)[0]
    print(json.dumps({"iters": iters, "E": E, "nonfinite_final": int(bad[-1].sum()),
                      "nonfinite_by_iter": [int(b) for b in bad.sum(1)],
                      "first_iters": {int(i): int(first[i]) for i in div[:200]}}))


if __name__ == "__main__":
    main()
