"""Loader for the C oracle of the TorchSDF kernels (oracle/sdf_oracle.c)."""
import ctypes as C
import os

import numpy as np

from tests.conftest import REPO

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(REPO, "oracle", "build", "libsdf_oracle.so")
        if not os.path.exists(path):
            from compliancedex_amd.build import build_oracle
            build_oracle()
        _lib = C.CDLL(path)
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def forward(points, faces):
    points = np.ascontiguousarray(points, np.float32)
    faces = np.ascontiguousarray(faces, np.float32).reshape(-1, 9)
    P, F = len(points), len(faces)
    d = np.zeros(P, np.float32); s = np.zeros(P, np.int32); n = np.zeros((P, 3), np.float32)
    c = np.zeros((P, 3), np.float32); f = np.zeros(P, np.int32)
    lib().sdf_oracle_forward(_p(points), C.c_int64(P), _p(faces), C.c_int64(F), _p(d), _p(s), _p(n), _p(c), _p(f))
    return d, s, n, c, f


def forward_f64(points, faces):
    points = np.ascontiguousarray(points, np.float64)
    faces = np.ascontiguousarray(faces, np.float64).reshape(-1, 9)
    P, F = len(points), len(faces)
    d = np.zeros(P, np.float64); s = np.zeros(P, np.int32); n = np.zeros((P, 3), np.float64)
    c = np.zeros((P, 3), np.float64); f = np.zeros(P, np.int32)
    lib().sdf_oracle_forward_f64(_p(points), C.c_int64(P), _p(faces), C.c_int64(F), _p(d), _p(s), _p(n), _p(c), _p(f))
    return d, s, n, c, f


def backward_f64(grad, points, clst):
    grad = np.ascontiguousarray(grad, np.float64)
    points = np.ascontiguousarray(points, np.float64)
    clst = np.ascontiguousarray(clst, np.float64)
    gp = np.zeros_like(points)
    lib().sdf_oracle_backward_f64(_p(grad), _p(points), _p(clst), C.c_int64(len(points)), _p(gp))
    return gp


def backward(grad, points, clst):
    grad = np.ascontiguousarray(grad, np.float32)
    points = np.ascontiguousarray(points, np.float32)
    clst = np.ascontiguousarray(clst, np.float32)
    gp = np.zeros_like(points)
    lib().sdf_oracle_backward(_p(grad), _p(points), _p(clst), C.c_int64(len(points)), _p(gp))
    return gp



def oracle_sdf(points, faces):
    """``sdf(points, faces)`` for the oracle loops: the C oracle's forward with the TorchSDF
    backward 2·g·(p − c) (sdf.py:56-64, .cu:256-270) as a torch autograd function on CPU tensors."""
    import torch

    class _Fn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, p, f):
            d, s, n, c, _ = forward(p.detach().numpy(), f.detach().numpy())
            ct = torch.from_numpy(c)
            ctx.save_for_backward(p.detach().clone(), ct)
            out = torch.from_numpy(d), torch.from_numpy(s), torch.from_numpy(n), ct
            ctx.mark_non_differentiable(*out[1:])
            return out

        @staticmethod
        def backward(ctx, gd, *_):
            p, c = ctx.saved_tensors
            return torch.from_numpy(backward(gd.contiguous().numpy(), p.numpy(), c.numpy())), None

    return _Fn.apply(points, faces)
