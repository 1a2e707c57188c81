"""Host check of csrc/svd3.h (the HOG kernel's per-point SVD) against numpy's
LAPACK dgesdd (fp64, as numpy runs it), which is what the reference runs (models/model_partseg.py:36-37):
compiles the header's host build with g++ and compares the dominant right
singular vector (sign included) and the singular value on random k x 3
neighbourhoods and on neighbourhoods gathered the way compute_hog_1x1 does.

  python tools/svd3_check.py [--trials 200000] [--k 20]
"""
import argparse
import ctypes
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
HDR = os.path.join(HERE, "..", "dgcnn.pytorch_amd", "csrc")

SHIM = r"""
#include "svd3.h"
extern "C" void svd3_batch(const float* A, int n, int k, float* s0, float* v) {
    double buf[4096];
    for (int p = 0; p < n; ++p) {
        for (int i = 0; i < 3 * k; ++i) buf[i] = A[(long)p * 3 * k + i];
        double vv[3], s;
        svd3::dominant_right_vector(buf, k, &s, vv);
        s0[p] = (float)s;
        for (int c = 0; c < 3; ++c) v[p * 3 + c] = (float)vv[c];
    }
}
"""


def build():
    d = tempfile.mkdtemp()
    src, so = os.path.join(d, "shim.cpp"), os.path.join(d, "shim.so")
    with open(src, "w") as f:
        f.write(SHIM)
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-I", HDR, src, "-o", so])
    lib = ctypes.CDLL(so)
    lib.svd3_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return lib


def run(lib, A):
    A = np.ascontiguousarray(A, np.float32)
    n, k, _ = A.shape
    s0 = np.zeros(n, np.float32)
    v = np.zeros((n, 3), np.float32)
    lib.svd3_batch(A.ctypes.data, n, k, s0.ctypes.data, v.ctypes.data)
    return s0, v


def compare(lib, A, label):
    s0, v = run(lib, A)
    _, S, Vh = np.linalg.svd(A, full_matrices=False)
    ref = Vh[:, 0, :]
    dot = np.einsum("nc,nc->n", v, ref)
    sign_ok = dot > 0
    gap = (S[:, 0] - S[:, 1]) / np.maximum(S[:, 0], 1e-30)
    well = gap > 1e-3
    err = np.abs(v - ref).max(1)
    print(f"{label}: n={len(A)} sign match {sign_ok.mean():.6f} (well-separated {sign_ok[well].mean():.6f},"
          f" {well.sum()} pts) | max |v - v_ref| (well) {err[well].max():.3e} | "
          f"max rel sigma err {np.max(np.abs(s0 - S[:, 0]) / S[:, 0]):.3e}")
    bad = np.nonzero(~sign_ok & well)[0]
    return bad


def hog_neighbourhoods(B, N, k, seed):
    """Neighbourhoods exactly as compute_hog_1x1 forms them: local kNN indices
    into the flat (B*N, 3) view of the contiguous (B, 3, N) tensor."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, 3, N)).astype(np.float32)
    inner = -2 * np.einsum("bcn,bcm->bnm", x, x)
    xx = (x ** 2).sum(1, keepdims=True)
    pd = -xx - inner - xx.transpose(0, 2, 1)
    idx = np.argsort(-pd, axis=-1, kind="stable")[:, :, :k]
    flat = x.reshape(B * N, 3)
    A = flat[idx[0]]
    return A - A.mean(1, keepdims=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=200000)
    ap.add_argument("--k", type=int, default=20)
    a = ap.parse_args()
    lib = build()
    rng = np.random.default_rng(0)
    for k in (a.k, 40, 5):
        A = rng.standard_normal((a.trials, k, 3)).astype(np.float32)
        A -= A.mean(1, keepdims=True)
        compare(lib, A, f"gaussian k={k}")
        A2 = A * np.array([3.0, 1.0, 0.01], np.float32)
        compare(lib, A2, f"anisotropic k={k}")
    bad = compare(lib, hog_neighbourhoods(4, 2048, a.k, 1), "hog neighbourhoods")
    if len(bad):
        print("first mismatches:", bad[:10])


if __name__ == "__main__":
    main()
