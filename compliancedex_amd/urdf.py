"""URDF → kinematic chain description (the data ``urdf_utils.py:12-126`` extracts).

A chain is a list of bodies in URDF link order (``robot_model.py:115-138``).  Each
body carries its parent index, the joint origin (xyz, rpy), the joint axis and type.
Controlled joints (type != fixed) get DOF indices in body order, exactly as the
reference numbers them (``robot_model.py:125-129``).
"""
from __future__ import annotations

import json
import os
import xml.etree.ElementTree as ET

_ROBOT_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "robots")


def _vec(s, default):
    if s is None:
        return list(default)
    v = [float(x) for x in s.split()]
    if len(v) != 3:
        raise ValueError(f"expected 3 floats, got {s!r}")
    return v


def parse_urdf(path):
    """Parses a URDF file into ``{"name", "bodies": [...]}``."""
    root = ET.parse(path).getroot()
    link_names = [el.get("name") for el in root if el.tag == "link"]
    joints = []
    for el in root:
        if el.tag != "joint":
            continue
        org = el.find("origin")
        ax = el.find("axis")
        lim = el.find("limit")
        joints.append(dict(
            name=el.get("name"), type=el.get("type"),
            parent=el.find("parent").get("link"), child=el.find("child").get("link"),
            xyz=_vec(org.get("xyz") if org is not None else None, (0, 0, 0)),
            rpy=_vec(org.get("rpy") if org is not None else None, (0, 0, 0)),
            axis=_vec(ax.get("xyz"), (1, 0, 0)) if ax is not None else [0.0, 0.0, 0.0],
            lower=float(lim.get("lower", 0)) if lim is not None else 0.0,
            upper=float(lim.get("upper", 0)) if lim is not None else 0.0,
        ))
    index = {n: i for i, n in enumerate(link_names)}
    bodies = []
    for i, name in enumerate(link_names):
        if i == 0:
            bodies.append(dict(name=name, parent=-1, joint="fixed", joint_name="base_joint",
                               xyz=[0.0] * 3, rpy=[0.0] * 3, axis=[0.0] * 3, lower=0.0, upper=0.0))
            continue
        # find_joint_of_body: first joint whose child is this link (urdf_utils.py:16-20)
        j = next((j for j in joints if j["child"] == name), None)
        if j is None:
            raise ValueError(f"link {name!r} has no parent joint")
        if index[j["parent"]] >= i:
            raise ValueError("URDF must list parents before children (robot_model.py:174-194)")
        fixed = j["type"] == "fixed"
        bodies.append(dict(name=name, parent=index[j["parent"]], joint="fixed" if fixed else j["type"],
                           joint_name=j["name"], xyz=j["xyz"], rpy=j["rpy"],
                           axis=[0.0] * 3 if fixed else j["axis"], lower=j["lower"], upper=j["upper"]))
    return dict(name=root.get("name", os.path.basename(path)), bodies=bodies)


def load_robot(name_or_path):
    """Loads a chain by packaged robot name (``allegro``, ``leap``, ``iiwa7_allegro``), a
    packaged JSON path, or a URDF path.  Packaged JSONs also carry the hand config
    (``*_hand_config.py``: ee links/offsets, ref_q, collision links/pairs)."""
    if os.path.exists(name_or_path):
        if name_or_path.endswith(".json"):
            with open(name_or_path) as f:
                return json.load(f)
        return parse_urdf(name_or_path)
    p = os.path.join(_ROBOT_DIR, f"{name_or_path}.json")
    if not os.path.exists(p):
        raise FileNotFoundError(f"no URDF or packaged robot named {name_or_path!r}")
    with open(p) as f:
        return json.load(f)


def dof_count(chain):
    return sum(1 for b in chain["bodies"][1:] if b["joint"] != "fixed")
