"""Packs a parsed kinematic chain into the ``cdx_chain`` descriptor (include/cdx.h)."""
from __future__ import annotations

import ctypes

import torch

from ._native import MAX_BODIES, MAX_DOFS, MAX_TIPS, CdxChain


def _axis_rot_f32(axis, angle):
    """Principal-axis rotation in float32, as x_rot/y_rot/z_rot (spatial_vector_algebra.py:14-53)."""
    a = torch.tensor([angle], dtype=torch.float32)
    c, s = torch.cos(a)[0], torch.sin(a)[0]
    R = torch.zeros(3, 3, dtype=torch.float32)
    if axis == 0:
        R[0, 0] = 1; R[1, 1] = c; R[1, 2] = -s; R[2, 1] = s; R[2, 2] = c
    elif axis == 1:
        R[0, 0] = c; R[0, 2] = s; R[1, 1] = 1; R[2, 0] = -s; R[2, 2] = c
    else:
        R[0, 0] = c; R[0, 1] = -s; R[1, 0] = s; R[1, 1] = c; R[2, 2] = 1
    return R


def fixed_rotation(rpy):
    """(Rz(yaw)·Ry(pitch))·Rx(roll) in float32 (rigid_body.py:138-144)."""
    r = torch.tensor(rpy, dtype=torch.float32)
    return (_axis_rot_f32(2, float(r[2])) @ _axis_rot_f32(1, float(r[1]))) @ _axis_rot_f32(0, float(r[0]))


def joint_axis(axis):
    """(axis id, sign) with the reference's recognition rule (rigid_body.py:149-155):
    |x| == 1 → x, elif |y| == 1 → y, else z with sign(z) (0 ⇒ the joint never moves)."""
    ax = torch.tensor(axis, dtype=torch.float32)
    if float(torch.abs(ax[0])) == 1:
        return 0, float(torch.sign(ax[0]))
    if float(torch.abs(ax[1])) == 1:
        return 1, float(torch.sign(ax[1]))
    return 2, float(torch.sign(ax[2]))


class Chain:
    """A robot's bodies with DOF numbering in URDF link order (robot_model.py:115-138)."""

    def __init__(self, desc):
        self.desc = desc
        self.bodies = desc["bodies"]
        if len(self.bodies) > MAX_BODIES:
            raise ValueError(f"chain has {len(self.bodies)} bodies; the descriptor holds {MAX_BODIES}")
        self.index = {b["name"]: i for i, b in enumerate(self.bodies)}
        self.dof = []
        n = 0
        for i, b in enumerate(self.bodies):
            if i > 0 and b["joint"] != "fixed":
                self.dof.append(n)
                n += 1
            else:
                self.dof.append(-1)
        self.n_dofs = n
        if n > MAX_DOFS:
            raise ValueError(f"chain has {n} DOFs; the descriptor holds {MAX_DOFS}")
        self._base = CdxChain()
        self._base.n_bodies = len(self.bodies)
        self._base.n_dofs = n
        for i, b in enumerate(self.bodies):
            cb = self._base.bodies[i]
            F = fixed_rotation(b["rpy"]).reshape(-1).tolist()
            for k in range(9):
                cb.F[k] = F[k]
            for k in range(3):
                cb.t[k] = float(torch.tensor(b["xyz"][k], dtype=torch.float32))
            ax, sg = joint_axis(b["axis"]) if self.dof[i] >= 0 else (2, 0.0)
            cb.axis, cb.sign = ax, sg
            cb.parent = b["parent"]
            cb.dof = self.dof[i]

    @property
    def config(self):
        return self.desc.get("config", {})

    def descriptor(self, link_names, offsets=None):
        """cdx_chain with the requested tips (and optional per-tip offsets)."""
        if len(link_names) > MAX_TIPS:
            raise ValueError(f"at most {MAX_TIPS} tips")
        if offsets is not None and len(offsets) != len(link_names):
            raise AssertionError("len(link_names) == len(offsets)")  # robot_model.py:242
        c = CdxChain()
        ctypes.memmove(ctypes.byref(c), ctypes.byref(self._base), ctypes.sizeof(c))
        c.n_tips = len(link_names)
        c.has_offsets = 1 if offsets is not None else 0
        for k, name in enumerate(link_names):
            if name not in self.index:
                raise KeyError(name)
            c.tip_body[k] = self.index[name]
            if offsets is not None:
                for i in range(3):
                    c.tip_offset[k][i] = float(torch.tensor(float(offsets[k][i]), dtype=torch.float32))
        return c
