"""In-tree build of the native libraries (no cmake/ninja; plain hipcc / g++ / gcc).

  compliancedex_amd/lib/libcdx.so        gfx950 kernels + C ABI (include/cdx.h) — the product
  compliancedex_amd/lib/libcdx_host.so   host build of the per-candidate code — CPU tests only
  oracle/build/libsdf_oracle.so          C oracle of the TorchSDF kernel — CPU tests only

``python -m compliancedex_amd.build`` or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
ARCH = os.environ.get("CDX_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["cdx_gpis.hip", "cdx_screen.hip", "cdx_fit.hip", "cdx_closure.hip", "cdx_sdf.hip", "cdx_optim.hip", "cdx_exchange.hip", "cdx_kin.hip"]
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _deps():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(REPO, "include", "cdx.h")]


# Tuning switches compiled into the product library.
DEFAULT_DEFINES = ("CDX_FAST_SQRT", "CDX_STD_SCHED", "CDX_MEAN_RSQ32")


def source_digest(defines=DEFAULT_DEFINES):
    """sha256 of what libcdx.so is compiled from: every file of csrc/ and include/cdx.h (by name and
    bytes, sorted), the -D switches and the offload arch."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted(_deps()):
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(("|".join(defines) + "|" + ARCH).encode())
    return h.hexdigest()


def _write_stamp(out, defines):
    with open(out + ".srcsha", "w") as f:
        f.write(source_digest(defines) + "\n")


def stamp_info(out=None, defines=DEFAULT_DEFINES):
    """{"src_sha16": digest of the tree's sources, "lib_sha16": the digest the library was built from
    (its .srcsha stamp, None if absent), "matches": both equal} — the library a run loads was built
    from exactly these sources (the GPU box runs the pushed binary without building)."""
    out = out or os.path.join(LIB, "libcdx.so")
    cur = source_digest(defines)
    try:
        with open(out + ".srcsha") as f:
            built = f.read().strip()
    except OSError:
        built = None
    return {"src_sha16": cur[:16], "lib_sha16": built[:16] if built else None, "matches": built == cur}


def build_device(force=False, defines=DEFAULT_DEFINES, out_name="libcdx.so"):
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, out_name)
    if not force and not _stale(out, _deps()):
        return out
    cmds, objs = [], []
    for src in HIP_SOURCES:
        obj = os.path.join(LIB, out_name + "." + src.replace(".hip", ".o"))
        # -Wno-pass-failed: `#pragma unroll` on loops whose trip count is only known at run time in the
        # runtime-fingertip-count instantiations (cdx_cost.h ForceEq<0>)
        flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-pass-failed", "-I",
                 os.path.join(REPO, "include")]
        flags += [f"-D{d}" for d in defines]
        # no FMA contraction in the per-candidate code (FK, Kabsch, costs) and TorchSDF: the
        # device then rounds like the reference's CPU float ops and like libcdx_host.so (the
        # collision cost's 1/d near the floor amplifies a contracted f32 FK to 1e-4)
        if src in ("cdx_sdf.hip", "cdx_closure.hip", "cdx_kin.hip"):
            flags.append("-ffp-contract=off")
        cmds.append([HIPCC, *flags, "-c", os.path.join(CSRC, src), "-o", obj])
        objs.append(obj)
    # one hipcc per translation unit, a few at a time (each holds ~1-2 GB while compiling)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(cmds), int(os.environ.get("CDX_BUILD_JOBS", "4"))))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, cmds))
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out])
    _write_stamp(out, defines)
    for o in objs:
        os.remove(o)
    return out


def build_host(force=False):
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, "libcdx_host.so")
    if not force and not _stale(out, _deps()):
        return out
    _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wno-unknown-pragmas",
          "-I", os.path.join(REPO, "include"), os.path.join(CSRC, "host_ref.cpp"), "-o", out])
    return out


def build_oracle(force=False):
    bdir = os.path.join(REPO, "oracle", "build")
    os.makedirs(bdir, exist_ok=True)
    src = os.path.join(REPO, "oracle", "sdf_oracle.c")
    out = os.path.join(bdir, "libsdf_oracle.so")
    if not force and not _stale(out, [src]):
        return out
    _run(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", src, "-o", out, "-lm"])
    return out


def build_all(force=False):
    return build_device(force), build_host(force), build_oracle(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
