"""compliancedex_amd — MI355X-native (gfx950) probabilistic-pregrasp inner loop of ComplianceDex.

Drop-in operators (same names / arguments as the reference):
  GPIS                         gpis.py:4-168
  DifferentiableRobotModel     differentiable_robot_model/robot_model.py (FK)
  compute_sdf                  torchsdf/sdf.py
  ProbabilisticGraspOptimizer  optimize_pregrasp.py:614-839
  KinGraspOptimizer / SDFGraspOptimizer / GPISGraspOptimizer / KinGPISGraspOptimizer
                               optimize_pregrasp.py:121-511
  force_eq_reward              optimize_pregrasp.py:73-118
All compute runs in libcdx.so (HIP, gfx950); importing works without a GPU, calling does not.
"""
from .gpis import GPIS  # noqa: F401
from .optimizer import (EE_OFFSETS, FINGERTIP_LB, FINGERTIP_UB, WRIST_OFFSET,  # noqa: F401
                        ProbabilisticGraspOptimizer, euler_angles_to_matrix)
from .anneal import PregraspAnnealer  # noqa: F401
from .force_eq import force_eq_reward  # noqa: F401
from .optimizers import (GPISGraspOptimizer, KinGPISGraspOptimizer, KinGraspOptimizer,  # noqa: F401
                         SDFGraspOptimizer, TriangleMesh)
from .robot_model import DifferentiableRobotModel  # noqa: F401
from .torchsdf import PreparedMesh, compute_sdf, compute_sdf_with_faces, index_vertices_by_faces  # noqa: F401

__version__ = "0.1.0"
