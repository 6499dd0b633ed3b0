"""Config 4's fused Kin loop (as tools/c4_divergence_gpu.py: config4_kin_inputs, the seed-7 float32 tape) run for
ITERS iterations, then the loop state of selected candidates dumped — the parameters the NEXT iteration would use
(q, target, compliance), Adam's moments, the step count — and the per-candidate losses of the run, so the CPU oracle
can take over from exactly that state (tests/test_gpu_configs.py::test_config4_divergence_state_injection's source).

  python tools/c4_state_dump.py ITERS cand,cand,...  →  gpurun_out/c4_state_<ITERS>.npz
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from compliancedex_amd import KinGraspOptimizer
    from compliancedex_amd.workloads import banana_mesh, config4_kin_inputs
    iters = int(sys.argv[1])
    cands = np.array([int(v) for v in sys.argv[2].split(",")])
    dev = torch.device("cuda:0")
    E = 16384
    links, offs, palm, q, target, comp = config4_kin_inputs(E, device=dev)
    tape = np.random.default_rng(7).random((iters, E, 3, 3), dtype=np.float32)
    noise = [torch.from_numpy(tape[s]).to(dev) for s in range(iters)]
    kin = KinGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=palm.tolist(), num_iters=iters,
                            optimize_target=True, ref_q=[0.0] * 23, device=dev)
    x = [torch.from_numpy(a).to(dev) for a in (q, target, comp)]
    kin.optimize(*x, 1, banana_mesh(), verbose=False, kabsch_noise=noise, trace_rows=True, fused=True)
    torch.cuda.synchronize()
    st = kin.last_loop
    c = torch.from_numpy(cands).to(dev)
    out = dict(cands=cands, iters=iters, palm=palm, loss=torch.stack(kin.loss_rows).cpu().numpy()[:, cands],
               q=st.pose[c].cpu().numpy(), target=st.target[c].cpu().numpy(), comp=st.comp[c].cpu().numpy(),
               m_q=st.m[0][c].cpu().numpy(), v_q=st.v[0][c].cpu().numpy(), m_t=st.m[1][c].cpu().numpy(),
               v_t=st.v[1][c].cpu().numpy(), m_c=st.m[2][c].cpu().numpy(), v_c=st.v[2][c].cpu().numpy(),
               tips=st.tips.view(E, 4, 3)[c].cpu().numpy())
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/c4_state_{iters}.npz", **out)
    print("dumped", iters, cands.tolist(), np.isfinite(out["q"]).all(1).tolist())


if __name__ == "__main__":
    main()
