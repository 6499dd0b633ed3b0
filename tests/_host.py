"""Test-only loader of libcdx_host.so (host build of the per-candidate device code)."""
import ctypes as C
import os

import numpy as np

from compliancedex_amd._native import LIB_DIR, CdxChain, CdxProblem

_lib = None


def host():
    global _lib
    if _lib is None:
        path = os.path.join(LIB_DIR, "libcdx_host.so")
        if not os.path.exists(path):
            from compliancedex_amd.build import build_host
            build_host()
        _lib = C.CDLL(path)
        P = C.c_void_p
        _lib.cdxh_n_queries.restype = C.c_int64
        _lib.cdxh_n_queries.argtypes = [C.POINTER(CdxProblem), C.c_int64]
    return _lib


def p(a):
    return a.ctypes.data_as(C.c_void_p)


def fk_forward(chain: CdxChain, q):
    q = np.ascontiguousarray(q, dtype=np.float32)
    B = q.shape[0]
    pos = np.zeros((B, chain.n_tips * 3), np.float32)
    quat = np.zeros((B, chain.n_tips * 4), np.float32)
    host().cdxh_fk_forward(C.byref(chain), p(q), C.c_int64(B), p(pos), p(quat))
    return pos, quat


def fk_backward(chain: CdxChain, q, gpos):
    q = np.ascontiguousarray(q, dtype=np.float32)
    gpos = np.ascontiguousarray(gpos, dtype=np.float32)
    gq = np.zeros_like(q)
    host().cdxh_fk_backward(C.byref(chain), p(q), C.c_int64(q.shape[0]), p(gpos), p(gq))
    return gq


def closure_queries(prob: CdxProblem, q, target, palm):
    E = q.shape[0]
    Mq = host().cdxh_n_queries(C.byref(prob), E)
    X = np.zeros((Mq, 3))
    q, target = np.ascontiguousarray(q, np.float64), np.ascontiguousarray(target, np.float64)
    pp, po = np.ascontiguousarray(palm[:, :3]), np.ascontiguousarray(palm[:, 3:])
    host().cdxh_closure_queries(C.byref(prob), C.c_int64(E), p(q), p(target), p(pp), p(po), p(X))
    return X


def closure_cost(prob: CdxProblem, q, comp, target, palm, noise, gp):
    E, D = q.shape
    T = prob.chain.n_tips
    K = prob.n_levels
    q, comp, target = [np.ascontiguousarray(a, np.float64) for a in (q, comp, target)]
    pp, po = np.ascontiguousarray(palm[:, :3]), np.ascontiguousarray(palm[:, 3:])
    noise = np.ascontiguousarray(noise, np.float64)
    out = dict(total_loss=np.zeros(E), total_margin=np.zeros((E, T)), grad_q=np.zeros((E, D)),
               grad_comp=np.zeros((E, T)), grad_target=np.zeros((E, T, 3)), grad_palm_pos=np.zeros((E, 3)),
               grad_palm_ori=np.zeros((E, 3)), flip=np.zeros(K * E, np.int32))
    arrs = [np.ascontiguousarray(gp[k], np.float64) for k in ("mean", "gmean", "normal", "std", "gstd")]
    host().cdxh_closure_cost(C.byref(prob), C.c_int64(E), p(q), p(comp), p(target), p(pp), p(po), p(noise),
                             *[p(a) for a in arrs],
                             *[p(out[k]) for k in ("total_loss", "total_margin", "grad_q", "grad_comp", "grad_target",
                                                   "grad_palm_pos", "grad_palm_ori", "flip")])
    return out


def svd3(H):
    H = np.ascontiguousarray(H, np.float64)
    U, S, V = np.zeros(9), np.zeros(3), np.zeros(9)
    host().cdxh_svd3(p(H), p(U), p(S), p(V))
    return U.reshape(3, 3), S, V.reshape(3, 3)


def sdf_forward(points, faces):
    points = np.ascontiguousarray(points, np.float32)
    faces = np.ascontiguousarray(faces, np.float32)
    P, F = len(points), len(faces)
    d = np.zeros(P, np.float32); s = np.zeros(P, np.int32); n = np.zeros((P, 3), np.float32)
    c = np.zeros((P, 3), np.float32); f = np.zeros(P, np.int32)
    host().cdxh_sdf_forward(p(points), C.c_int64(P), p(faces), C.c_int64(F), p(d), p(s), p(n), p(c), p(f))
    return d, s, n, c, f


def collision(desc, q, palm):
    q = np.ascontiguousarray(q, np.float64)
    pp, po = np.ascontiguousarray(palm[:, :3]), np.ascontiguousarray(palm[:, 3:])
    E, D = q.shape
    cost, g_q = np.zeros(E), np.zeros((E, D))
    g_pp, g_po = np.zeros((E, 3)), np.zeros((E, 3))
    host().cdxh_collision(C.byref(desc), C.c_int64(E), p(q), p(pp), p(po), p(cost), p(g_q), p(g_pp), p(g_po))
    return cost, g_q, np.concatenate([g_pp, g_po], 1)


def force_eq(desc, tip, target, comp, normal, noise, g_reward, g_fn):
    B, T = comp.shape
    a = [np.ascontiguousarray(x, np.float64) for x in (tip, target, comp, normal, noise, g_reward, g_fn)]
    reward, margin, fn = np.zeros(B), np.zeros((B, T)), np.zeros((B, T))
    flip = np.zeros(B, np.int32)
    g_tip, g_target, g_comp = np.zeros((B, T, 3)), np.zeros((B, T, 3)), np.zeros((B, T))
    host().cdxh_force_eq(C.byref(desc), C.c_int64(B), *(p(x) for x in a), p(reward), p(margin), p(fn), p(flip),
                         p(g_tip), p(g_target), p(g_comp))
    return dict(reward=reward, margin=margin, force_norm=fn, flip=flip, grad_tip=g_tip, grad_target=g_target,
                grad_comp=g_comp)
