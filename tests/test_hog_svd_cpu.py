"""f1 host check: csrc/svd3.h (the per-point SVD inside dgx_hog_1x1_f32) built
for the host with g++ reproduces np.linalg.svd's dominant right singular vector
and singular value — sign included — on the neighbourhoods compute_hog_1x1 forms
(reference models/model_partseg.py:28-37). numpy runs LAPACK dgesdd in fp64 on
the fp32 input and rounds to fp32; the restatement follows the same routine
path, so the fp32 results are identical, not just close."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

SHIM = r"""
#include "svd3.h"
extern "C" void svd3_batch(const float* A, int n, int k, float* s0, float* v) {
    double buf[3 * 64];
    for (int p = 0; p < n; ++p) {
        for (int i = 0; i < 3 * k; ++i) buf[i] = A[(long)p * 3 * k + i];
        double vv[3], s;
        svd3::dominant_right_vector(buf, k, &s, vv);
        s0[p] = (float)s;
        for (int c = 0; c < 3; ++c) v[p * 3 + c] = (float)vv[c];
    }
}
"""


@pytest.fixture(scope="module")
def svd3(tmp_path_factory):
    d = tmp_path_factory.mktemp("svd3")
    src, so = d / "shim.cpp", d / "shim.so"
    src.write_text(SHIM)
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-I",
                           os.path.join(REPO, "dgcnn.pytorch_amd", "csrc"), str(src), "-o", str(so)])
    lib = ctypes.CDLL(str(so))
    lib.svd3_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]

    def run(A):
        A = np.ascontiguousarray(A, np.float32)
        n, k, _ = A.shape
        s0, v = np.zeros(n, np.float32), np.zeros((n, 3), np.float32)
        lib.svd3_batch(A.ctypes.data, n, k, s0.ctypes.data, v.ctypes.data)
        return s0, v
    return run


def _hog_neighbourhoods(rng, B, N, k):
    # the reference's local-id gather over the (B*N, 3) view, cloud 0's rows
    import oracle
    x = rng.standard_normal((B, 3, N)).astype(np.float32)
    idx = oracle.knn(x, k)
    A = x.reshape(B * N, 3)[idx[0]]
    return (A - A.mean(axis=1, keepdims=True, dtype=np.float32)).astype(np.float32)


@pytest.mark.parametrize("k", [5, 10, 20, 40, 64])
def test_svd3_matches_numpy(svd3, k):
    rng = np.random.default_rng(k)
    A = rng.standard_normal((4000, k, 3)).astype(np.float32)
    A -= A.mean(axis=1, keepdims=True)
    A[:1000] *= np.array([5.0, 1.0, 1e-3], np.float32)          # strongly anisotropic
    A[1000:1100] = 0.0                                           # zero neighbourhoods
    A[1100:1200] = A[1100:1200, :, :1] * np.array([1.0, -2.0, 0.5], np.float32)  # rank 1
    s0, v = svd3(A)
    _, S, Vh = np.linalg.svd(A, full_matrices=False)
    np.testing.assert_array_equal(v, Vh[:, 0, :])
    np.testing.assert_array_equal(s0, S[:, 0])


def test_svd3_on_hog_neighbourhoods(svd3):
    A = _hog_neighbourhoods(np.random.default_rng(1), 2, 1024, 20)
    s0, v = svd3(A)
    _, S, Vh = np.linalg.svd(A, full_matrices=False)
    np.testing.assert_array_equal(v, Vh[:, 0, :])
    np.testing.assert_array_equal(s0, S[:, 0])
