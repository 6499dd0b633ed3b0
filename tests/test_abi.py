"""The C-ABI library loads (no GPU needed) and exports every symbol include/cdx.h declares;
binding struct layouts match the library's sizeof.  CPU only."""
import os
import re

from tests.conftest import REPO


def declared_functions():
    src = open(os.path.join(REPO, "include", "cdx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(cdx_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_path():
    names = declared_functions()
    for n in ("cdx_gpis_mean", "cdx_gpis_std", "cdx_fk_forward", "cdx_fk_backward", "cdx_closure",
              "cdx_sdf_forward", "cdx_sdf_backward"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from compliancedex_amd import _native
    lib = _native.load()  # also checks struct sizes against the library
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.cdx_version().startswith(b"compliancedex_amd")


def test_shipped_library_ignores_ab_switches():
    """the shipped libcdx.so is built without -DCDX_AB_SWITCHES, so CDX_SCREEN_AUDIT / CDX_SCREEN_REPAIR /
    CDX_NO_SCREEN and the schedule switches in a user's environment are ignored (csrc/cdx_ab.h); the default build's
    -D list carries no A/B switch.  (tests/test_screen.py::test_env_switches_cannot_disable_the_repair runs the
    closure with them set on the GPU.)"""
    from compliancedex_amd import _native
    from compliancedex_amd.build import DEFAULT_DEFINES
    assert _native.load().cdx_ab_switches() == 0
    assert "CDX_AB_SWITCHES" not in DEFAULT_DEFINES


def test_bad_arguments_are_rejected_without_launch():
    import ctypes
    from compliancedex_amd import _native as N
    lib = N.load()
    g = N.CdxGpis()
    assert lib.cdx_gpis_mean(g, None, 10, None, None, None, None) == -1
    g.kernel = 7
    g.X1 = g.alpha = 1
    g.N, g.N_pad = 1, 64
    assert lib.cdx_gpis_mean(g, None, 10, None, None, None, None) == -2
    c = N.CdxChain()
    assert lib.cdx_fk_forward(c, None, 1, None, None, None) == -3
    assert lib.cdx_sdf_forward(None, 5, None, 0, None, None, None, None, None, None) == -1
    assert lib.cdx_sdf_query(None, None, 0, None, 5, None, None, None, None, None, None, 0, 0, None) == -1
    assert lib.cdx_sdf_query_workspace(0) == 0 and lib.cdx_sdf_mesh_bytes(0) == 0
    assert lib.cdx_sdf_mesh_prepare(None, 10, None, None) == -1
    assert lib.cdx_sdf_query_order(None, 5, None, 0, None) == -1 and lib.cdx_sdf_query_order(None, -1, None, 0, None) == -1
    assert lib.cdx_sdf_query_batch(5, None, None, 0, None) == -1 and lib.cdx_sdf_query_batch(1, None, None, 0, None) == -1
    q = N.CdxSdfBatchQuery()
    q.P, q.F, q.flags = 10, 4, N.SDF_REUSE_ORDER  # (not marked culled)
    assert lib.cdx_sdf_query_batch(1, ctypes.cast(ctypes.pointer(q), ctypes.c_void_p), None, 0, None) == -1
    # the launch schedule: 4 header words, then a duration and an order slot per 64-point group
    Ps = (ctypes.c_int64 * 3)(65536, 65536, 100)
    assert lib.cdx_sdf_batch_schedule_bytes(3, Ps) == 4 * (4 + 2 * (1024 + 1024 + 2))
    assert lib.cdx_sdf_batch_schedule_bytes(5, Ps) == 0 and lib.cdx_sdf_batch_schedule_bytes(1, None) == 0
    cfg, buf = N.CdxKinOpt(), N.CdxKinOptBuffers()
    cfg.rule = 2
    assert lib.cdx_kin_step(None, cfg, buf, 4, 4, 0, 0, None) == -1  # unknown rule
    cfg.rule = 0
    assert lib.cdx_kin_step(None, cfg, buf, 4, 4, 0, 0, None) == -1  # Adam (Kin) without a chain
    cfg.rule = 1
    assert lib.cdx_kin_step(None, cfg, buf, 4, 4, 0, 0, None) == -1  # null buffers
    prm = N.CdxKinParams()
    prm.fe.n_tips = 4
    assert lib.cdx_kin_iteration(None, None, cfg, buf, 4, 4, *[None] * 10, 0, 0, None) == -1  # no params
    cfg.rule = 0
    assert lib.cdx_kin_iteration(None, prm, cfg, buf, 4, 4, *[None] * 10, 0, 0, None) == -1  # Kin without a chain
    assert lib.cdx_kin_iteration(c, prm, cfg, buf, 4, 3, *[None] * 10, 0, 0, None) == -1  # tip count mismatch
    # the FK-walk cache: one block of (12 + 6·16 + 8 + 4) slots × 64 lanes of floats per 64-lane workgroup (four lanes
    # a candidate), none for other fingertip counts or no candidates
    assert lib.cdx_kin_fk_state_bytes(16384, 4) == 1024 * 120 * 64 * 4
    assert lib.cdx_kin_fk_state_bytes(3000, 4) == 188 * 120 * 64 * 4
    assert lib.cdx_kin_fk_state_bytes(3000, 3) == 0 and lib.cdx_kin_fk_state_bytes(0, 4) == 0
    p = N.CdxProblem()
    assert lib.cdx_closure_workspace(p, 10) == 0
    assert lib.cdx_closure(p, 10, *([None] * 6), ctypes.c_uint64(0), *([None] * 11)) == -1


def test_product_refuses_cpu_tensors():
    import pytest
    import torch
    from compliancedex_amd import GPIS
    g = GPIS(0.08, 1.0)
    g.load_state_data("banana_state", device="cpu")
    with pytest.raises(RuntimeError, match="no CPU path"):
        g.pred(torch.zeros(4, 3, dtype=torch.float64))


def test_batch_schedule_host_logic():
    """torchsdf.BatchSchedule (host side of cdx_sdf_query_batch's schedule): sized by cdx_sdf_batch_schedule_bytes,
    zeroed when (re)allocated, the order recomputed on every `every`-th launch and whenever the group count changes."""
    import torch
    from compliancedex_amd.torchsdf import BatchSchedule
    dev = torch.device("cpu")
    sch = BatchSchedule(every=4)
    buf = sch.get([65536, 65536, 100], dev)
    assert buf.numel() == 4 * (4 + 2 * (1024 + 1024 + 2)) and int(buf.sum()) == 0
    keeps = [sch.keep_order() for _ in range(9)]
    assert keeps == [False, True, True, True, False, True, True, True, False]
    sch.get([6000, 6000, 3000], dev)  # fewer groups: the same buffer, the order recomputed next
    assert sch.buf is buf and sch.keep_order() is False and sch.keep_order() is True
    big = sch.get([1 << 20], dev)  # more groups than the buffer holds: a new, zeroed buffer
    assert big is not buf and big.numel() == 4 * (4 + 2 * 16384) and sch.keep_order() is False
