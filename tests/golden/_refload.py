"""Container-only loader that imports the ComplianceDex reference in-process on CPU.

Used ONLY by ``make_golden.py`` to generate the committed golden fixtures.  It never
ships, and nothing under ``tests/`` imports it at test time (``/root/reference`` does
not exist on the GPU box).

What it does:
  * ``PYTORCH_JIT=0`` so the two ``@torch.jit.script`` helpers on the path
    (``optimize_pregrasp.py:49`` ``optimal_transformation_batch`` and
    ``se3_so3_util.py:240`` ``quat_rotate``) run as plain Python, where the
    hard-coded ``.cuda()`` calls can be neutralised.
  * ``torch.Tensor.cuda`` -> identity (the path pins ``cuda:0`` everywhere).
  * Stub modules for imports that are not on the hot path and are absent here:
    ``open3d`` (visualisation), ``torchsdf`` (its ``_C.so`` blob is missing),
    ``pybullet`` (simulation), ``cvxpy`` / ``cvxpylayers`` (WC optimiser only),
    and ``pybullet_robot.robots`` (its ``__init__`` imports pybullet; we load the two
    ``*_config.py`` data files by path instead).
  * ``urdf_parser_py`` is not installed: a data-only XML reader provides the fields
    ``urdf_utils.py:12-126`` reads (links, joints: name/type/parent/child/origin
    xyz+rpy/axis/limit).  Inertial data is reported as absent (FK does not use it).
  * ``DifferentiableRobotModel`` is forced onto the CPU device.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types
import xml.etree.ElementTree as ET

REF = os.environ.get("CDX_REFERENCE", "/root/reference")


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(mod, k, v)
    sys.modules[name] = mod
    return mod


class _Obj:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _floats(s, n, default):
    if s is None:
        return list(default)
    vals = [float(v) for v in s.split()]
    assert len(vals) == n
    return vals


def _urdf_from_xml_file(path):
    root = ET.parse(path).getroot()
    links, joints = [], []
    for el in root:
        if el.tag == "link":
            links.append(_Obj(name=el.get("name"), inertial=None))
        elif el.tag == "joint":
            org = el.find("origin")
            origin = _Obj(
                position=_floats(org.get("xyz") if org is not None else None, 3, (0, 0, 0)),
                rotation=_floats(org.get("rpy") if org is not None else None, 3, (0, 0, 0)),
            )
            ax = el.find("axis")
            lim = el.find("limit")
            dyn = el.find("dynamics")
            joints.append(_Obj(
                name=el.get("name"), type=el.get("type"),
                parent=el.find("parent").get("link"), child=el.find("child").get("link"),
                origin=origin,
                axis=_floats(ax.get("xyz"), 3, (1, 0, 0)) if ax is not None else None,
                limit=_Obj(effort=float(lim.get("effort", 0)), lower=float(lim.get("lower", 0)),
                           upper=float(lim.get("upper", 0)), velocity=float(lim.get("velocity", 0)))
                if lim is not None else None,
                dynamics=_Obj(damping=float(dyn.get("damping", 0))) if dyn is not None else None,
            ))
    return _Obj(links=links, joints=joints)


_LOADED = None


def load():
    """Returns a namespace with the reference modules (gpis, optimize_pregrasp, robot model)."""
    global _LOADED
    if _LOADED is not None:
        return _LOADED
    os.environ["PYTORCH_JIT"] = "0"
    import torch  # noqa: E402
    import numpy as np  # noqa: F401

    torch.Tensor.cuda = lambda self, *a, **k: self

    _stub("open3d")
    _stub("torchsdf", compute_sdf=None)
    _stub("pybullet")
    _stub("cvxpy")
    _stub("cvxpylayers")
    _stub("cvxpylayers.torch", CvxpyLayer=None)
    up = _stub("urdf_parser_py")
    upu = _stub("urdf_parser_py.urdf", URDF=_Obj(from_xml_file=_urdf_from_xml_file))
    up.urdf = upu

    robots_dir = os.path.join(REF, "pybullet_robot/src/pybullet_robot/robots")
    cfgs = {}
    for hand, rel in (("allegro", "allegro_hand/allegro_hand_config.py"),
                      ("leap", "leap_hand/leap_hand_config.py")):
        spec = importlib.util.spec_from_file_location(f"_cfg_{hand}", os.path.join(robots_dir, rel))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        cfgs[hand] = m.ROBOT_CONFIG
    pr = _stub("pybullet_robot")
    prr = _stub("pybullet_robot.robots", robot_configs=cfgs)
    pr.robots = prr

    import matplotlib
    matplotlib.use("Agg")

    for p in (REF, os.path.join(REF, "thirdparty/differentiable-robot-model")):
        if p not in sys.path:
            sys.path.insert(0, p)

    from differentiable_robot_model import robot_model as rm  # noqa: E402
    _orig_init = rm.DifferentiableRobotModel.__init__

    def _cpu_init(self, urdf_path, name="", device=None):
        _orig_init(self, urdf_path, name=name, device="cpu")

    rm.DifferentiableRobotModel.__init__ = _cpu_init

    import gpis as ref_gpis  # noqa: E402
    import optimize_pregrasp as ref_opt  # noqa: E402

    _LOADED = _Obj(torch=torch, gpis=ref_gpis, opt=ref_opt, rm=rm, robot_configs=cfgs, ref=REF)
    return _LOADED


URDFS = {
    "allegro": "pybullet_robot/src/pybullet_robot/robots/allegro_hand/models/allegro_hand_description_left.urdf",
    "leap": "pybullet_robot/src/pybullet_robot/robots/leap_hand/assets/leap_hand/robot.urdf",
    "iiwa7_allegro": "thirdparty/differentiable-robot-model/diff_robot_data/kuka_iiwa/urdf/iiwa7_allegro.urdf",
}
