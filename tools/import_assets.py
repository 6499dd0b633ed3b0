"""Container-only: packs the reference's DATA files the hot path needs into the package.

  compliancedex_amd/robots/<robot>.json   URDF → chain (our parser) + hand config values
                                          (allegro_hand_config.py:3-28, leap_hand_config.py:3-28)
  compliancedex_amd/data/gpis_states/<obj>_state.npz   stored GPIS states (gpis.py:155-168 format)
  compliancedex_amd/data/meshes/<obj>_faces.npy        face_vertices [F,3,3] float32 (banana mesh,
                                          TorchSDF test models cube / sphere-42)
  compliancedex_amd/data/meshes/banana_mesh.npz        banana vertices (f64) + triangles
  compliancedex_amd/data/banana_center.npy, partial_pcd_banana.npy
  compliancedex_amd/data/config3_surface.npz           config 3's N = 2000 GPIS surfaces: 1 936 points per
                                          object sampled area-weighted from assets/<obj>/<obj>.obj
                                          (hammer, lego, mug, mug2) or drawn from the observed point
                                          cloud (assets/coffeebottle/completed_pcd.npz), seeded

Run: ``python tools/import_assets.py`` (reads /root/reference; the GPU box never needs it).
"""
from __future__ import annotations

import ast
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from compliancedex_amd.urdf import parse_urdf  # noqa: E402

REF = os.environ.get("CDX_REFERENCE", "/root/reference")
PKG = os.path.join(REPO, "compliancedex_amd")

URDFS = {
    "allegro": "pybullet_robot/src/pybullet_robot/robots/allegro_hand/models/allegro_hand_description_left.urdf",
    "leap": "pybullet_robot/src/pybullet_robot/robots/leap_hand/assets/leap_hand/robot.urdf",
    "iiwa7_allegro": "thirdparty/differentiable-robot-model/diff_robot_data/kuka_iiwa/urdf/iiwa7_allegro.urdf",
}
CONFIGS = {
    "allegro": "pybullet_robot/src/pybullet_robot/robots/allegro_hand/allegro_hand_config.py",
    "leap": "pybullet_robot/src/pybullet_robot/robots/leap_hand/leap_hand_config.py",
}


def read_config(path):
    """Evaluates the ROBOT_CONFIG dict literal (numpy arrays / np.pi only) without importing it."""
    src = open(path).read()
    tree = ast.parse(src)
    for node in tree.body:
        if isinstance(node, ast.Assign) and node.targets[0].id == "ROBOT_CONFIG":
            expr = ast.Expression(node.value)
            val = eval(compile(expr, path, "eval"), {"np": np, "__builtins__": {}})
            return {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in val.items()}
    raise ValueError(path)


def obj_faces(path):
    vs, fs = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                vs.append([float(x) for x in line.split()[1:4]])
            elif line.startswith("f "):
                fs.append([int(tok.split("/")[0]) - 1 for tok in line.split()[1:4]])
    vs, fs = np.asarray(vs, dtype=np.float64), np.asarray(fs)
    return vs, fs


def sample_surface(vs, fs, n, rng):
    """Area-weighted uniform samples on a triangle mesh."""
    tri = vs[fs]
    area = 0.5 * np.linalg.norm(np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]), axis=1)
    pick = rng.choice(len(fs), n, p=area / area.sum())
    u, v = rng.random(n), rng.random(n)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    t = tri[pick]
    return t[:, 0] + u[:, None] * (t[:, 1] - t[:, 0]) + v[:, None] * (t[:, 2] - t[:, 0])


def config3_surfaces(n=1936):
    rng = np.random.default_rng(3)
    out = {}
    for obj in ("hammer", "lego", "mug", "mug2"):
        vs, fs = obj_faces(os.path.join(REF, "assets", obj, f"{obj}.obj"))
        out[obj] = sample_surface(vs, fs, n, rng)
    obs = np.load(os.path.join(REF, "assets/coffeebottle/completed_pcd.npz"))["observed"]
    out["coffeebottle"] = obs[rng.choice(len(obs), n, replace=False)].astype(np.float64)
    np.savez_compressed(os.path.join(PKG, "data", "config3_surface.npz"), **out)
    print("config3 surfaces", {k: v.shape for k, v in out.items()})


def main():
    if sys.argv[1:] == ["config3"]:
        return config3_surfaces()
    os.makedirs(os.path.join(PKG, "robots"), exist_ok=True)
    for robot, rel in URDFS.items():
        chain = parse_urdf(os.path.join(REF, rel))
        chain["name"] = robot
        if robot in CONFIGS:
            chain["config"] = read_config(os.path.join(REF, CONFIGS[robot]))
        else:
            chain["config"] = {"ee_link_name": ["link_3.0_tip", "link_7.0_tip", "link_11.0_tip", "link_15.0_tip"]}
        with open(os.path.join(PKG, "robots", f"{robot}.json"), "w") as f:
            json.dump(chain, f, indent=1)
        print("robot", robot, len(chain["bodies"]))

    gdir = os.path.join(PKG, "data", "gpis_states")
    os.makedirs(gdir, exist_ok=True)
    for obj in ["banana", "coffeebottle", "hammer", "lego", "mug", "mug2", "dummy"]:
        shutil.copyfile(os.path.join(REF, "gpis_states", f"{obj}_state.npz"), os.path.join(gdir, f"{obj}_state.npz"))

    mdir = os.path.join(PKG, "data", "meshes")
    os.makedirs(mdir, exist_ok=True)
    meshes = {"banana": "assets/banana/banana.obj",
              "cube": "thirdparty/TorchSDF/tests/models/cube.obj",
              "sphere42": "thirdparty/TorchSDF/tests/models/sphere-42.obj"}
    for name, rel in meshes.items():
        vs, fs = obj_faces(os.path.join(REF, rel))
        np.save(os.path.join(mdir, f"{name}_faces.npy"), vs[fs].astype(np.float32))
        if name == "banana":  # f64 vertices + triangles: the SDF optimisers rescale the mesh (:163-164)
            np.savez_compressed(os.path.join(mdir, f"{name}_mesh.npz"), vertices=vs, triangles=fs.astype(np.int32))
            np.save(os.path.join(PKG, "data", "banana_center.npy"), 0.5 * (vs.min(0) + vs.max(0)))
        print("mesh", name, fs.shape)
    shutil.copyfile(os.path.join(REF, "partial_pcd/banana.npy"), os.path.join(PKG, "data", "partial_pcd_banana.npy"))
    config3_surfaces()


if __name__ == "__main__":
    main()
