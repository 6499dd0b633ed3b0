"""Optimiser results in the reference's on-disk format.

Writer: optimize_pregrasp.py:1016-1020 saves five float64 arrays per experiment under data/:
  contact_<exp>.npy [E,4,3] (fingertips at the optimum: forward_kinematics(q, palm), :1009),
  target_<exp>.npy [E,4,3], wrist_<exp>.npy [E,6], compliance_<exp>.npy [E,4],
  joint_angle_<exp>.npy [E,16].
Readers: verify_pregrasp.py:147-155 (contact / target / compliance), verify_grasp_robot.py:150-154.
"""
from __future__ import annotations

import os

import numpy as np

NAMES = ("contact", "target", "wrist", "compliance", "joint_angle")


def _np(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def save_results(exp_name, contact, target, wrist, compliance, joint_angle, data_dir="data"):
    os.makedirs(data_dir, exist_ok=True)
    paths = []
    for name, arr in zip(NAMES, (contact, target, wrist, compliance, joint_angle)):
        path = os.path.join(data_dir, f"{name}_{exp_name}.npy")
        np.save(path, _np(arr))
        paths.append(path)
    return paths


def load_results(exp_name, data_dir="data"):
    return {name: np.load(os.path.join(data_dir, f"{name}_{exp_name}.npy")) for name in NAMES}


def optimize_and_save(optimizer, gpis, init_joint_angles, target_pose, compliance, exp_name, friction_mu=1,
                      data_dir="data", **kw):
    """optimize → FK of the optimum → save, as optimize_pregrasp.py:1008-1020 does (headless)."""
    q, comp, target, palm, margin = optimizer.optimize(init_joint_angles, target_pose, compliance, friction_mu, gpis,
                                                       **kw)
    contact = optimizer.forward_kinematics(q, palm)
    save_results(exp_name, contact, target, palm, comp, q, data_dir)
    return dict(joint_angle=q, compliance=comp, target=target, wrist=palm, margin=margin, contact=contact)
