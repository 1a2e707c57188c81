"""TEST INFRASTRUCTURE ONLY — CPU oracle for the EdgeConv hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this package, and only as the checker. The product path
(``dgcnn.pytorch_amd/dgx``, ``libdgx.so``) never imports it; with the HIP
library missing the product raises instead of falling back here.

Contents
  * ``knn`` / ``sqnorm`` / ``pairwise`` — ctypes bindings of ``knn_oracle.c``, the
    bit-exact fp32 restatement of reference ``models/dgcnn.py:6-12``.
  * ``graph_feature`` — numpy restatement of ``models/dgcnn.py:15-44``.
  * ``reference.py`` — torch-CPU restatement of the float path (EdgeConv blocks,
    DGCNN, PositionEmbedding) used for 1e-3 parity and as the CPU baseline.
  * ``hog.hog_1x1`` — torch/numpy-CPU restatement of compute_hog_1x1 after its
    kNN call (models/model_partseg.py:28-92).

Pinned by ``tests/golden/`` fixtures that ``tests/golden/make_goldens.py``
produced by running the reference itself in the build container.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_knn.so")
_lib = None

ORDER_STRIDED = 0  # x**2 laid out N-contiguous: torch's strided (cascade-16) reduction
ORDER_VEC8X4 = 1   # x**2 laid out C-contiguous: torch's vectorised inner reduction


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        i64, i32, vp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
        lib.oracle_sqnorm.argtypes = [vp, i64, i64, i64, i32, i32, i32, i32, vp]
        lib.oracle_sqnorm.restype = None
        lib.oracle_pairwise.argtypes = [vp, i64, i64, i64, i32, i32, i32, i32, vp]
        lib.oracle_pairwise.restype = None
        lib.oracle_knn.argtypes = [vp, i64, i64, i64, i32, i32, i32, i32, i32, vp, vp]
        lib.oracle_knn.restype = ctypes.c_int
        _lib = lib
    return _lib


def reduction_order(shape, strides):
    """Which torch CPU reduction order ``sum(x**2, dim=1)`` takes for a (B,C,N)
    tensor of these element strides (x**2 inherits x's layout when x is dense)."""
    _, C, N = shape
    _, sC, sN = strides
    if C > 1 and N > 1 and sC < sN:
        return ORDER_VEC8X4
    return ORDER_STRIDED


def _as_view(x):
    """(array, element strides) for a float32 numpy array or CPU torch tensor,
    keeping its layout (so the oracle sees what the reference would)."""
    try:
        import torch
        if isinstance(x, torch.Tensor):
            x = x.detach()
            assert x.dtype == torch.float32 and x.device.type == "cpu"
            return x, tuple(x.stride()), x.data_ptr()
    except ImportError:
        pass
    x = np.asarray(x)
    assert x.dtype == np.float32
    strides = tuple(s // 4 for s in x.strides)
    return x, strides, x.ctypes.data


def sqnorm(x, order=None):
    x, (sB, sC, sN), ptr = _as_view(x)
    B, C, N = x.shape
    if order is None:
        order = reduction_order(x.shape, (sB, sC, sN))
    out = np.empty((B, N), np.float32)
    _load().oracle_sqnorm(ptr, sB, sC, sN, B, C, N, order, out.ctypes.data)
    return out


def pairwise(x, order=None):
    """(B,N,N) pd exactly as reference dgcnn.py:7-9 computes it."""
    x, (sB, sC, sN), ptr = _as_view(x)
    B, C, N = x.shape
    if order is None:
        order = reduction_order(x.shape, (sB, sC, sN))
    out = np.empty((B, N, N), np.float32)
    _load().oracle_pairwise(ptr, sB, sC, sN, B, C, N, order, out.ctypes.data)
    return out


def knn(x, k, order=None, return_values=False):
    """Canonical-order kNN (pd desc, index asc): int64 (B,N,k), reference dgcnn.py:6-12."""
    x, (sB, sC, sN), ptr = _as_view(x)
    B, C, N = x.shape
    if order is None:
        order = reduction_order(x.shape, (sB, sC, sN))
    idx = np.empty((B, N, k), np.int64)
    vals = np.empty((B, N, k), np.float32)
    rc = _load().oracle_knn(ptr, sB, sC, sN, B, C, N, k, order,
                            idx.ctypes.data, vals.ctypes.data)
    if rc != 0:
        raise RuntimeError("selected index k out of range")
    return (idx, vals) if return_values else idx


def canonicalize(idx, pd):
    """Re-order a (B,N,k) index set into canonical order (value desc, index asc)
    given the full pd matrix — used to compare with torch.topk's arbitrary ties."""
    B, N, k = idx.shape
    vals = np.take_along_axis(pd, idx, axis=2)
    order = np.lexsort((idx, -vals), axis=-1)
    return np.take_along_axis(idx, order, axis=2), np.take_along_axis(vals, order, axis=2)


def graph_feature(x, idx, knn_only=False, disp_only=False):
    """numpy restatement of reference dgcnn.py:15-44 given the neighbour indices.

    x (B,C,N) float32, idx (B,N,k) local indices. Default output (B,2C,N,k) with
    channels [0,C) = x_j (neighbour) and [C,2C) = x_i (centre), dgcnn.py:42.
    knn_only -> (B,N,k,C) neighbour rows (dgcnn.py:37-38); disp_only -> (B,C,N,k)
    x_j - x_i (dgcnn.py:39-40)."""
    x = np.asarray(x, np.float32)
    B, C, N = x.shape
    pts = np.ascontiguousarray(x.transpose(0, 2, 1))           # (B,N,C)
    nbr = pts[np.arange(B)[:, None, None], idx]                  # (B,N,k,C)
    if knn_only:
        return nbr
    ctr = np.broadcast_to(pts[:, :, None, :], nbr.shape)
    if disp_only:
        return np.ascontiguousarray((nbr - ctr).transpose(0, 3, 1, 2))
    return np.ascontiguousarray(np.concatenate([nbr, ctr], axis=3).transpose(0, 3, 1, 2))
