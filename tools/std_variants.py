"""A/B timing of gpis_std_kernel build variants (one process per variant, same inputs).

  python tools/std_variants.py build            # builds lib/libcdx_<name>.so for each variant (CPU)
  python tools/std_variants.py run [M] [N]      # on the GPU: times cdx_gpis_std for each built variant

Times the whitened std pass alone (gpis_std(..., want_grad=False): the triangular K*·L⁻ᵀ GEMM +
finalize); TFLOPs counts the useful M·N(N+1).  The nogen / nomfma builds are timing-only
diagnostics (their outputs are wrong): they bound the cost of the on-chip K* generation and of the
MFMA issue.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
VARIANTS = {"wn4": ("CDX_FAST_SQRT", "CDX_STD_SCHED"),               # default build
            "wn4_nosched": ("CDX_FAST_SQRT",),
            "gensqrtfull": ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_GEN_SQRT_FULL"),  # full sqrt in K* generation
            "kload": ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_VAR_KLOAD"),  # whitened pass reads a K* buffer
            "nodiag": ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_STD_NODIAG"),  # no diagonal-block MFMA trimming
            "old2buf": None,                                       # prebuilt older library, not rebuilt
            "diag_nogen": ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_DIAG_NOGEN"),
            "diag_nomfma": ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_DIAG_NOMFMA"),
            "diag_nobload": ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_DIAG_NOBLOAD"),
            "diag_wgtime": ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_DIAG_WGTIME"),
            "diag_nobload_nogen": ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_DIAG_NOBLOAD", "CDX_DIAG_NOGEN")}
if os.environ.get("CDX_VARIANTS"):  # e.g. CDX_VARIANTS=wn4,t4_nosched
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in os.environ["CDX_VARIANTS"].split(",")}


def build():
    from compliancedex_amd.build import build_device
    for name, defs in VARIANTS.items():
        if defs is None:
            continue
        build_device(force=True, defines=defs, out_name=f"libcdx_{name}.so")


def child(lib, M, N, ref_path):
    os.environ["CDX_LIB"] = lib
    import numpy as np
    import torch
    from compliancedex_amd.gpis import gpis_std
    from compliancedex_amd.workloads import synthetic_banana_gpis
    g = synthetic_banana_gpis(N, "cuda")
    st = g.native_state()
    X1 = g.X1.cpu().numpy()
    rng = np.random.default_rng(0)
    lo, hi = X1.min(0) - 0.03, X1.max(0) + 0.03
    X = torch.from_numpy(lo + (hi - lo) * rng.random((M, 3))).cuda()
    for _ in range(3):
        std, _ = gpis_std(st, X, want_grad=False)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 20
    ev[0].record()
    for _ in range(reps):
        std, _ = gpis_std(st, X, want_grad=False)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    # with ∇std: + the GRADV pass (E11⁻¹k = L⁻ᵀv from the kept V) for all M queries
    for _ in range(2):
        gpis_std(st, X, want_grad=True)
    ev[0].record()
    for _ in range(reps):
        gpis_std(st, X, want_grad=True)
    ev[1].record()
    torch.cuda.synchronize()
    ms_grad = ev[0].elapsed_time(ev[1]) / reps - ms
    out = std.unsqueeze(1).cpu().numpy()
    if "wgtime" in lib:  # per-workgroup timeline of one whitened pass (CDX_DIAG_WGTIME builds)
        import ctypes
        from compliancedex_amd import _native
        gpis_std(st, X, want_grad=False)
        torch.cuda.synchronize()
        n = 16384
        buf = np.zeros((n, 4), dtype=np.uint64)
        _native.load().cdx_diag_wgtime.argtypes = [ctypes.c_void_p, ctypes.c_int]
        assert _native.load().cdx_diag_wgtime(buf.ctypes.data, n) == 0
        np.save(os.path.join(REPO, "gpurun_out", f"wgtime_{M}_{N}.npy"), buf)
    if not os.path.exists(ref_path):
        np.save(ref_path, out)
    ref = np.load(ref_path)
    err = float(np.abs(out - ref).max() / np.abs(ref).max())
    tf = M * float(N) * (N + 1) / (ms * 1e-3) / 1e12
    print(json.dumps({"lib": os.path.basename(lib), "M": M, "N": N, "ms": ms, "TFLOPs": tf, "rel_diff_vs_first": err,
                      "gradv_ms": ms_grad, "gradv_TFLOPs": tf * ms / ms_grad}))


def run(M, N):
    ref = os.path.join(REPO, "gpurun_out", f"std_ref_{M}_{N}.npy")
    if os.path.exists(ref):
        os.remove(ref)
    for name in VARIANTS:
        lib = os.path.join(REPO, "compliancedex_amd", "lib", f"libcdx_{name}.so")
        if os.path.exists(lib):
            subprocess.run([sys.executable, __file__, "child", lib, str(M), str(N), ref], check=True, timeout=300)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    elif sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 16384, int(sys.argv[3]) if len(sys.argv) > 3 else 2000)
    else:
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
