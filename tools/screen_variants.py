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
            "sub1": BASE + ("CDX_SC_SUB=1",),  # 16-K stages (one barrier per 16 K rows)
            "ring3": BASE + ("CDX_SC_RING=3",),  # 32-K stages, B DMA'd two stages ahead (160 KB LDS)
            "prio_young": BASE + ("CDX_SC_PRIO_YOUNG",),  # s_setprio 1 for waves 4-7 before the loop
            "pp": BASE + ("CDX_SC_PP=1",),  # ping-pong: the two waves of a SIMD multiply in alternate half-stages
            "w4": BASE + ("CDX_SC_WAVES=4",),  # 4 waves of 128 x 128 (one per SIMD, AGPR accumulators)
            "w4_sub1": BASE + ("CDX_SC_WAVES=4", "CDX_SC_SUB=1"),
            "w16": BASE + ("CDX_SC_WAVES=16",),  # 16 waves of 64 x 64 (four per SIMD, <= 128 registers)
            "w16_ring3": BASE + ("CDX_SC_WAVES=16", "CDX_SC_RING=3"),
            "diag_noread": BASE + ("CDX_SC_DIAG_NOREAD",),      # MFMAs on fragments read once per stage
            "diag_nobar": BASE + ("CDX_SC_DIAG_NOBAR",),        # no s_barrier in the loop (races)
            "diag_nodma": BASE + ("CDX_SC_DIAG_NODMA",),        # no B DMAs in the loop
            "diag_nogen": BASE + ("CDX_SC_DIAG_NOGEN",),
            "diag_nomfma": BASE + ("CDX_SC_DIAG_NOMFMA",),
            "diag_nogen_nomfma": BASE + ("CDX_SC_DIAG_NOGEN", "CDX_SC_DIAG_NOMFMA"),
            # MFMAs only: fragments from lane ids, no generation, no B DMA, no barrier
            "diag_mfma_only": BASE + ("CDX_SC_DIAG_NOREAD", "CDX_SC_DIAG_NOGEN", "CDX_SC_DIAG_NODMA", "CDX_SC_DIAG_NOBAR"),
            "diag_noepi": BASE + ("CDX_SC_DIAG_NOEPI",),  # no epilogue (Σ (Ṽ + c)² through LDS)
            "epireg": BASE + ("CDX_SC_EPI_REG=1",),  # epilogue summed from the accumulator registers
            "epilds": BASE + ("CDX_SC_EPI_REG=0",),  # epilogue through the LDS image
            "diag_noread_nogen": BASE + ("CDX_SC_DIAG_NOREAD", "CDX_SC_DIAG_NOGEN"),
            "diag_noread_nodma": BASE + ("CDX_SC_DIAG_NOREAD", "CDX_SC_DIAG_NODMA")}
# measured and dropped (profiles/r02j_screen_variants.jsonl): sched_group_barrier 1 MFMA : 6 VALU
# interleave (+10 %), s_setprio 1 around the MFMA block (+6 %).  Round 3 (profiles/r03j-l_*): B staged
# through VGPRs + ds_write instead of LDS-DMA (+1 %); row-block order with A-fragment prefetch (+2 %);
# X1 rows loaded one sub-step ahead (+4 %); both with a 1 MFMA : 4 VALU sched_group_barrier pipeline
# (+4..9 %); X1 rows not loaded at all (diagnostic, ±0); a register-A kernel (each wave 32 rows × 256
# columns, Ã generated in registers, only B through LDS, B ring of 2/3/4 by asm LDS-DMA) +4..6 %.
if os.environ.get("CDX_VARIANTS"):
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in os.environ["CDX_VARIANTS"].split(",")}


def build():
    """Only cdx_screen.hip differs between variants: the other objects are compiled once."""
    import shutil
    import tempfile
    from compliancedex_amd import build as B
    tmp = tempfile.mkdtemp(prefix="cdx_sc_")
    common = []
    for src in B.HIP_SOURCES:
        if src == "cdx_screen.hip":
            continue
        obj = os.path.join(tmp, src.replace(".hip", ".o"))
        extra = ["-ffp-contract=off"] if src in ("cdx_sdf.hip", "cdx_closure.hip") else []
        B._run([B.HIPCC, *_flags(B, BASE), *extra, "-c", os.path.join(B.CSRC, src), "-o", obj])
        common.append(obj)
    for name, defs in VARIANTS.items():
        obj = os.path.join(tmp, f"screen_{name}.o")
        B._run([B.HIPCC, *_flags(B, defs), "-c", os.path.join(B.CSRC, "cdx_screen.hip"), "-o", obj])
        B._run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *common, obj, "-o",
                os.path.join(B.LIB, f"libcdx_sc_{name}.so")])
    shutil.rmtree(tmp)


def _flags(B, defs):
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={B.ARCH}", "-Wno-pass-failed", "-I",
            os.path.join(REPO, "include")] + [f"-D{d}" for d in defs]


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
    from compliancedex_amd.gpis import exact_var
    est0 = st.screen_var(X)
    err = float((est0 - exact_var(st, X)).abs().max()) / float(g.R) ** 3
    repeat_equal = all(torch.equal(est0, st.screen_var(X)) for _ in range(20))
    import hashlib
    digest = hashlib.sha256(est0.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.path.basename(lib), "M": M, "screen_ms": ms, "max_err_over_k0": err, "bitwise_repeatable": repeat_equal, "estimate_sha256": digest,
                      "f16_tflops": 3 * M * 2000 * 2001 / ms / 1e9}), flush=True)


def run(E):
    for name in list(VARIANTS) * int(os.environ.get("CDX_VARIANT_ROUNDS", "1")):
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
