"""A/B timing of gpis_screen_kernel build variants (one process per variant, same inputs).

  python tools/screen_variants.py build        # lib/libcdx_sc_<name>.so per variant (CPU)
  python tools/screen_variants.py run [E]      # on the GPU: screen_var time per variant (JSON lines)

The diag_* builds are timing-only diagnostics (outputs wrong): they bound the cost of the fp32 K*
generation + split, of the B-slice loads, and of the MFMA issue.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
BASE = ("CDX_FAST_SQRT", "CDX_STD_SCHED")
VARIANTS = {"base": BASE,
            "diag_nogen": BASE + ("CDX_SC_DIAG_NOGEN",),
            "diag_nomfma": BASE + ("CDX_SC_DIAG_NOMFMA",),
            "diag_nogen_nomfma": BASE + ("CDX_SC_DIAG_NOGEN", "CDX_SC_DIAG_NOMFMA")}
# measured and dropped (profiles/r02j_screen_variants.jsonl): sched_group_barrier 1 MFMA : 6 VALU
# interleave (+10 %), s_setprio 1 around the MFMA block (+6 %)
if os.environ.get("CDX_VARIANTS"):
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in os.environ["CDX_VARIANTS"].split(",")}


def build():
    from compliancedex_amd.build import build_device
    for name, defs in VARIANTS.items():
        build_device(force=True, defines=defs, out_name=f"libcdx_sc_{name}.so")


def child(lib, E):
    os.environ["CDX_LIB"] = lib
    import torch
    from tools.screen_bench import alltip_queries, timed
    from compliancedex_amd.workloads import synthetic_banana_gpis
    g = synthetic_banana_gpis(2000, device="cuda")
    st = g.native_state()
    X = alltip_queries(E).cuda()
    ms = timed(lambda: st.screen_var(X), 20)
    M = X.shape[0]
    print(json.dumps({"lib": os.path.basename(lib), "M": M, "screen_ms": ms,
                      "bf16_tflops": 6 * M * 2000 * 2001 / ms / 1e9}), flush=True)


def run(E):
    for name in VARIANTS:
        lib = os.path.join(REPO, "compliancedex_amd", "lib", f"libcdx_sc_{name}.so")
        if os.path.exists(lib):
            subprocess.run([sys.executable, __file__, "child", lib, str(E)], check=False, timeout=300)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    elif sys.argv[1] == "child":
        child(sys.argv[2], int(sys.argv[3]))
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 4096)
