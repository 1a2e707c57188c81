"""a1 parity on adversarial coordinate clouds (reference models/dgcnn.py:6-12
on DGCNN block 1's xyz input, models/layers.py:45, models/model_partseg.py:26):
the engine kNN against the CPU oracle, bit for bit — tight clusters far apart,
lone outliers, all points identical (every distance ties), ShapeNet-like
surface clouds, lattice points (ties at every k), 1- and 2-channel clouds and
both input layouts; the int32 and int64 outputs agree."""
import numpy as np
import pytest
import torch

import oracle
from conftest import assert_knn_equivalent
from dgx import synth

pytestmark = pytest.mark.gpu


def _knn(x, k):
    from dgx.ops import knn_raw
    idx, vals = knn_raw(x, k, return_values=True)
    i32 = knn_raw(x, k, out_dtype=torch.int32)
    assert torch.equal(idx.to(torch.int32), i32)
    return idx, vals


def _clouds(kind, B, N, seed):
    rng = np.random.default_rng(seed)
    if kind == "cube":
        return synth.cube_clouds(B, N, seed)
    if kind == "clusters":   # two tight clusters 1e3 apart: the grid's cells are mostly empty
        x = rng.normal(scale=1e-3, size=(B, N, 3)).astype(np.float32)
        x[:, N // 2:, 0] += 1e3
        return x
    if kind == "outliers":   # a unit cloud plus a few points far away (their kNN leave any box)
        x = synth.cube_clouds(B, N, seed)
        x[:, :5] *= np.float32(50.0)
        return x
    if kind == "same":       # every point identical: all distances tie
        return np.full((B, N, 3), 0.25, np.float32)
    if kind == "surface":    # points on a sphere and a plane (ShapeNet-like: 2-D density in 3-D)
        a = rng.normal(size=(B, N // 2, 3))
        a /= np.linalg.norm(a, axis=-1, keepdims=True)
        p = np.concatenate([rng.uniform(-1, 1, (B, N - N // 2, 2)), np.full((B, N - N // 2, 1), -1.0)], -1)
        return np.concatenate([a, p], 1).astype(np.float32)
    if kind == "grid":       # lattice points: many exact distance ties at every k
        n = int(round(N ** (1 / 3))) + 1
        g = np.stack(np.meshgrid(*[np.arange(n)] * 3, indexing="ij"), -1).reshape(-1, 3)[:N]
        return np.broadcast_to(g.astype(np.float32) * np.float32(0.125), (B, N, 3)).copy()
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["cube", "clusters", "outliers", "same", "surface", "grid"])
@pytest.mark.parametrize("N,k", [(1024, 20), (2048, 40), (300, 64), (4096, 20), (57, 57), (200, 7)])
def test_knn_adversarial_clouds(cuda, kind, N, k):
    B = 2
    pts = _clouds(kind, B, N, N + k)
    f = torch.from_numpy(pts).permute(0, 2, 1)
    gi, gv = _knn(f.to(cuda), k)
    ref_idx, ref_vals = oracle.knn(f, k, return_values=True)
    np.testing.assert_array_equal(gv.cpu().numpy(), ref_vals)
    np.testing.assert_array_equal(gi.cpu().numpy(), ref_idx)


@pytest.mark.parametrize("C", [1, 2, 3])
@pytest.mark.parametrize("layout", ["bcn", "perm"])
def test_knn_channels_and_layouts(cuda, C, layout):
    """1-, 2- and 3-channel clouds, channel-major (B,C,N) and the permuted
    (B,N,C) view main_cls.py:91 feeds: equal to the oracle in the reference's
    rounding order of |x|^2 for that layout."""
    B, N, k = 3, 777, 16
    pts = synth.cube_clouds(B, N, 40 + C)[..., :C].copy()
    f = torch.from_numpy(pts).permute(0, 2, 1)
    if layout == "bcn":
        f = f.contiguous()
    x = f.to(cuda)
    gi, gv = _knn(x, k)
    ref_idx, ref_vals = oracle.knn(f, k, return_values=True)
    assert_knn_equivalent(gi.cpu().numpy(), gv.cpu().numpy(), ref_idx, ref_vals)
    np.testing.assert_array_equal(gi.cpu().numpy(), ref_idx)


def test_knn_is_deterministic(cuda):
    """Repeated launches give bitwise-identical outputs (surface cloud, k 40)."""
    x = torch.from_numpy(_clouds("surface", 4, 2048, 3)).to(cuda).permute(0, 2, 1)
    a = _knn(x, 40)
    for _ in range(3):
        b = _knn(x, 40)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
