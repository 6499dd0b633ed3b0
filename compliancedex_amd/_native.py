"""ctypes binding of the C ABI in ``include/cdx.h`` (libcdx.so, gfx950).

There is no CPU fallback: if the library is missing or fails to load, every operator
raises.  Struct layouts are checked against the library's own ``sizeof`` at load time.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")

MAX_BODIES, MAX_TIPS, MAX_DOFS, MAX_LEVELS = 32, 8, 32, 4
KERNELS = {"tps": 0, "rbf": 1, "joint": 2}
NPAD_ALIGN = 256  # CDX_NPAD_ALIGN
SCREEN_BANDS = 24  # CDX_SCREEN_BANDS
PROF_STAGES = 6   # cdx_profile_read array length
SDF_REUSE_ORDER, SDF_MESH_CULLED, SDF_MESH_EXACT = 1, 2, 4  # cdx_sdf_query flags
SDF_SCHED_KEEP = 8  # cdx_sdf_query_batch, first query: keep the schedule's order
ERRORS = {-1: "invalid argument", -2: "unsupported GPIS kernel", -3: "chain exceeds descriptor capacity",
          -10: "HIP launch failed"}


class CdxGpis(C.Structure):
    _fields_ = [("X1", C.c_void_p), ("alpha", C.c_void_p), ("Ainv", C.c_void_p), ("Linv_t", C.c_void_p),
                ("Linv", C.c_void_p), ("N", C.c_int32),
                ("N_pad", C.c_int32), ("kernel", C.c_int32), ("_pad", C.c_int32), ("R", C.c_double),
                ("sigma", C.c_double), ("bias", C.c_double), ("screen", C.c_void_p), ("screen_delta", C.c_double)]


class CdxBody(C.Structure):
    _fields_ = [("F", C.c_float * 9), ("t", C.c_float * 3), ("sign", C.c_float), ("axis", C.c_int8),
                ("parent", C.c_int8), ("dof", C.c_int8), ("_pad", C.c_int8)]


class CdxChain(C.Structure):
    _fields_ = [("n_bodies", C.c_int32), ("n_dofs", C.c_int32), ("n_tips", C.c_int32), ("has_offsets", C.c_int32),
                ("tip_body", C.c_int32 * MAX_TIPS), ("tip_offset", (C.c_float * 3) * MAX_TIPS),
                ("bodies", CdxBody * MAX_BODIES)]


class CdxProblem(C.Structure):
    _fields_ = [("chain", CdxChain), ("gpis", CdxGpis), ("n_levels", C.c_int32), ("n_query_levels", C.c_int32),
                ("level_query", C.c_int32 * MAX_LEVELS), ("coeff", (C.c_float * MAX_TIPS) * MAX_LEVELS),
                ("weight", C.c_double * MAX_LEVELS), ("ref_q", C.c_float * MAX_DOFS), ("cos_mu", C.c_float),
                ("gravity", C.c_int32), ("optimize_palm", C.c_int32), ("_pad", C.c_int32), ("com", C.c_float * 3),
                ("dummy_target_z", C.c_float), ("dummy_comp", C.c_float), ("_pad2", C.c_float),
                ("uncertainty", C.c_double), ("loop", C.c_void_p)]


MAX_PAIRS = 28


class CdxCollision(C.Structure):
    _fields_ = [("chain", CdxChain), ("n_pairs", C.c_int32), ("palm_term", C.c_int32),
                ("pairs", (C.c_int8 * 2) * MAX_PAIRS), ("pair_threshold", C.c_double), ("floor_z", C.c_double)]


class CdxForceEq(C.Structure):
    _fields_ = [("cos_mu", C.c_float), ("gravity", C.c_int32), ("com", C.c_float * 3), ("dummy_target_z", C.c_float),
                ("dummy_comp", C.c_float), ("n_tips", C.c_int32)]


class CdxKinParams(C.Structure):
    _fields_ = [("fe", CdxForceEq), ("ref_q", C.c_float * MAX_DOFS)]


class CdxKinOpt(C.Structure):
    _fields_ = [("rule", C.c_int32), ("clamp_box", C.c_int32), ("lr", C.c_double * 3), ("beta1", C.c_double),
                ("beta2", C.c_double), ("eps", C.c_double), ("alpha", C.c_double), ("palm_offset", C.c_float * 3),
                ("box_lb", C.c_float * (MAX_TIPS * 3)), ("box_ub", C.c_float * (MAX_TIPS * 3)), ("_pad", C.c_int32)]


KIN_OPT_FIELDS = ["pose", "target", "comp", "g_pose", "g_target", "g_comp", "m_pose", "v_pose", "m_target", "v_target",
                  "m_comp", "v_comp", "loss"]


class CdxKinOptBuffers(C.Structure):
    _fields_ = ([(n, C.c_void_p) for n in KIN_OPT_FIELDS] + [("margin", C.c_void_p * 2), ("normal", C.c_void_p * 2)] +
                [(n, C.c_void_p) for n in ("opt_value", "opt_margin", "opt_normal", "opt_pose", "opt_target",
                                            "opt_comp", "any", "tips", "fk_state")])


class CdxSdfBatchQuery(C.Structure):
    _fields_ = [("mesh", C.c_void_p), ("faces", C.c_void_p), ("F", C.c_int64), ("points", C.c_void_p), ("P", C.c_int64),
                ("sqdist", C.c_void_p), ("sign", C.c_void_p), ("normals", C.c_void_p), ("clst", C.c_void_p),
                ("face_idx", C.c_void_p), ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t),
                ("flags", C.c_int32), ("_pad", C.c_int32)]


class CdxAdam(C.Structure):
    _fields_ = [("lr", C.c_double * 5), ("beta1", C.c_double), ("beta2", C.c_double), ("eps", C.c_double),
                ("comp_min", C.c_double), ("target_lb", C.c_double * (MAX_TIPS * 3)),
                ("target_ub", C.c_double * (MAX_TIPS * 3)), ("clamp_target", C.c_int32), ("best_after", C.c_int32)]


OPT_BUFFER_FIELDS = ["q", "comp", "target", "palm_pos", "palm_ori", "g_q", "g_comp", "g_target", "g_palm_pos",
                     "g_palm_ori", "m_q", "v_q", "m_comp", "v_comp", "m_target", "v_target", "m_palm_pos",
                     "v_palm_pos", "m_palm_ori", "v_palm_ori", "total_loss", "total_margin", "opt_value", "opt_margin",
                     "opt_q", "opt_comp", "opt_target", "opt_palm"]


class CdxOptBuffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in OPT_BUFFER_FIELDS] + [("loop", C.c_void_p)]


class CdxScreenReport(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("screened", "screened_rows", "exact_rows", "audited_rows", "bound_misses",
                                         "audit_misses", "audit_flips", "faults")] + \
               [("max_ratio", C.c_double), ("max_ratio_audit", C.c_double)] + \
               [(n, C.c_int64) for n in ("cum_closures", "cum_audited_rows", "cum_bound_misses", "cum_audit_misses",
                                         "cum_audit_flips", "cum_faults")] + \
               [("cum_max_ratio", C.c_double), ("cum_max_ratio_audit", C.c_double)] + \
               [("repaired", C.c_int32), ("discarded_rows", C.c_int32), ("min_gap", C.c_double),
                ("audit_cut", C.c_double), ("cum_repairs", C.c_int64), ("cum_discarded_rows", C.c_int64),
                ("cum_min_gap", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_P = C.c_void_p
_I64 = C.c_int64
_SIGS = {
    "cdx_gpis_mean": (C.c_int, [C.POINTER(CdxGpis), _P, _I64, _P, _P, _P, _P]),
    "cdx_gpis_std_workspace": (C.c_size_t, [C.POINTER(CdxGpis), _I64]),
    "cdx_gpis_std": (C.c_int, [C.POINTER(CdxGpis), _P, _I64, _P, _P, _P, _P]),
    "cdx_gpis_screen_bytes": (C.c_size_t, [C.c_int32]),
    "cdx_gpis_screen_prepare": (C.c_int, [C.POINTER(CdxGpis), _P, _P]),
    "cdx_gpis_screen_set_bands": (C.c_int, [C.POINTER(CdxGpis), C.POINTER(C.c_double), _P]),
    "cdx_gpis_screen_info": (C.c_int, [C.POINTER(CdxGpis), C.POINTER(C.c_double), _P]),
    "cdx_gpis_screen_workspace": (C.c_size_t, [C.POINTER(CdxGpis), _I64]),
    "cdx_gpis_screen_var": (C.c_int, [C.POINTER(CdxGpis), _P, _I64, _P, _P, _P]),
    "cdx_gpis_fit": (C.c_int, [_P, C.c_int32, _P, C.c_int32, C.c_double, _P, _P, _P]),
    "cdx_gpis_factor_workspace": (C.c_size_t, [C.c_int32]),
    "cdx_gpis_factor": (C.c_int, [_P, _P, C.c_int32, C.c_int32, _P, _P, _P, _P, _P, _P, _P]),
    "cdx_fk_forward": (C.c_int, [C.POINTER(CdxChain), _P, _I64, _P, _P, _P]),
    "cdx_fk_backward": (C.c_int, [C.POINTER(CdxChain), _P, _I64, _P, _P, _P]),
    "cdx_force_eq_forward": (C.c_int, [C.POINTER(CdxForceEq), _I64, _P, _P, _P, _P, _P, C.c_uint64, _P, _P, _P, _P,
                                       _P]),
    "cdx_force_eq_backward": (C.c_int, [C.POINTER(CdxForceEq), _I64, _P, _P, _P, _P, _P, C.c_uint64, _P, _P, _P, _P,
                                        _P, _P]),
    "cdx_collision_loss": (C.c_int, [C.POINTER(CdxCollision), _I64, _P, _P, _P, _P, _P, _P, _P, C.c_int32, _P]),
    "cdx_closure_workspace": (C.c_size_t, [C.POINTER(CdxProblem), _I64]),
    "cdx_closure_screen_stats": (C.c_int, [C.POINTER(CdxProblem), _I64, _P, C.POINTER(C.c_int32)]),
    "cdx_closure_screen_report": (C.c_int, [C.POINTER(CdxProblem), _I64, _P, C.POINTER(CdxScreenReport), _P]),
    "cdx_closure_screen_reset": (C.c_int, [C.POINTER(CdxProblem), _I64, _P, _P]),
    "cdx_debug_fail_next_closure": (C.c_int, [C.c_int32]),
    "cdx_ab_switches": (C.c_int, []),
    "cdx_closure": (C.c_int, [C.POINTER(CdxProblem), _I64, _P, _P, _P, _P, _P, _P, C.c_uint64, _P,
                              _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cdx_pack_survivors": (C.c_int, [_I64, C.c_int32, C.c_int32, _P, _P, _P, _P, _P, _P, C.c_double, C.c_double,
                                     _I64, _I64, _P, _P]),
    "cdx_sdf_forward": (C.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "cdx_sdf_backward": (C.c_int, [_P, _P, _P, _I64, _P, _P]),
    "cdx_sdf_forward_f64": (C.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "cdx_sdf_backward_f64": (C.c_int, [_P, _P, _P, _I64, _P, _P]),
    "cdx_sdf_stats": (C.c_int, [C.c_int32, C.POINTER(C.c_uint64), _P]),
    "cdx_sdf_chunk_visits": (C.c_int, [C.POINTER(C.c_uint64), _P]),
    "cdx_kin_cost": (C.c_int, [C.POINTER(CdxChain), C.POINTER(CdxKinParams), _I64] + [_P] * 14 + [C.c_uint64] +
                     [_P] * 8),
    "cdx_sdf_mesh_bytes": (C.c_size_t, [_I64]),
    "cdx_sdf_mesh_prepare": (C.c_int, [_P, _I64, _P, _P]),
    "cdx_sdf_query_workspace": (C.c_size_t, [_I64]),
    "cdx_sdf_query_order": (C.c_int, [_P, _I64, _P, C.c_size_t, _P]),
    "cdx_sdf_batch_schedule_bytes": (C.c_size_t, [C.c_int32, _P]),
    "cdx_sdf_query_batch": (C.c_int, [C.c_int32, _P, _P, C.c_size_t, _P]),
    "cdx_sdf_query": (C.c_int, [_P, _P, _I64, _P, _I64, _P, _P, _P, _P, _P, _P, C.c_size_t, C.c_int32, _P]),
    "cdx_sdf_mesh_flags": (C.c_int, [_P, C.POINTER(C.c_int32), _P]),
    "cdx_version": (C.c_char_p, []),
    "cdx_abi_sizes": (None, [C.POINTER(C.c_size_t)]),
    "cdx_selftest_mfma_f64": (C.c_int, [_P, _P, _P, _P]),
    "cdx_profile_enable": (C.c_int, [C.c_int]),
    "cdx_optimizer_step": (C.c_int, [C.POINTER(CdxAdam), C.POINTER(CdxOptBuffers), _I64, C.c_int32, C.c_int32,
                                     C.c_int32, _P]),
    "cdx_profile_read": (C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "cdx_kin_step": (C.c_int, [C.POINTER(CdxChain), C.POINTER(CdxKinOpt), C.POINTER(CdxKinOptBuffers), _I64, C.c_int32,
                               C.c_int32, C.c_int32, _P]),
    "cdx_kin_fk_state_bytes": (_I64, [_I64, C.c_int32]),
    "cdx_kin_iteration": (C.c_int, [C.POINTER(CdxChain), C.POINTER(CdxKinParams), C.POINTER(CdxKinOpt),
                                    C.POINTER(CdxKinOptBuffers), _I64, C.c_int32] + [_P] * 10 +
                          [C.c_uint64, C.c_int32, _P]),
}

_lib = None
_lock = threading.Lock()


def lib_path():
    return os.environ.get("CDX_LIB", os.path.join(LIB_DIR, "libcdx.so"))


def load():
    """Loads libcdx.so (raises ImportError if it is missing — there is no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        if not os.path.exists(path):
            raise ImportError(f"compliancedex_amd native library not built: {path} "
                              "(run `python -m compliancedex_amd.build`)")
        lib = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        sizes = (C.c_size_t * 13)()
        lib.cdx_abi_sizes(sizes)
        mine = [C.sizeof(CdxGpis), C.sizeof(CdxBody), C.sizeof(CdxChain), C.sizeof(CdxProblem),
                C.sizeof(CdxCollision), C.sizeof(CdxAdam), C.sizeof(CdxOptBuffers), C.sizeof(CdxForceEq),
                C.sizeof(CdxScreenReport), C.sizeof(CdxKinParams), C.sizeof(CdxKinOpt), C.sizeof(CdxKinOptBuffers),
                C.sizeof(CdxSdfBatchQuery)]
        if list(sizes) != mine:
            raise ImportError(f"ABI struct size mismatch: library {list(sizes)} vs binding {mine}")
        info = build_info()
        if not info["matches"] and "CDX_LIB" not in os.environ:
            import warnings
            warnings.warn(f"{path} was not built from this tree's csrc/ (stamp {info['lib_sha16']}, sources "
                          f"{info['src_sha16']}): rebuild with `python -m compliancedex_amd.build`")
        _lib = lib
        return lib


def build_info():
    """Source digest of the tree vs the one libcdx.so was built from (build.stamp_info)."""
    from .build import stamp_info
    return stamp_info(lib_path())


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {ERRORS.get(rc, rc)} (code {rc})")


def ptr(t):
    """Device pointer of a (contiguous) tensor, or None."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return t.data_ptr()


def stream_ptr(device=None):
    import torch
    return torch.cuda.current_stream(device).cuda_stream
