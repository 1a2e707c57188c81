"""a1 parity: dgx kNN (HIP) vs the reference's goldens and the CPU oracle."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN, assert_knn_equivalent
from dgx import synth

pytestmark = pytest.mark.gpu

KNN_CASES = ["c3", "c9", "c64", "c128", "c3k40", "c64k32", "c3n1000"]


def _view(pts, layout, dev):
    t = torch.from_numpy(pts).to(dev)
    return t.permute(0, 2, 1) if layout == "perm" else t.permute(0, 2, 1).contiguous()


def _cpu_view(pts, layout):
    t = torch.from_numpy(pts)
    return t.permute(0, 2, 1) if layout == "perm" else t.permute(0, 2, 1).contiguous()


@pytest.mark.parametrize("layout", ["bcn", "perm"])
@pytest.mark.parametrize("case", KNN_CASES)
def test_knn_matches_reference_golden(golden, cuda, case, layout):
    from models.dgcnn import knn
    g = golden("knn_cases.npz")
    key = f"{case}_{layout}"
    k = g[key + "_idx"].shape[-1]
    idx = knn(_view(g[key + "_x"], layout, cuda), k)
    assert idx.dtype == torch.int64 and tuple(idx.shape) == g[key + "_idx"].shape
    np.testing.assert_array_equal(idx.cpu().numpy(), g[key + "_idx"])


def test_knn_ties_golden(golden, cuda):
    from models.dgcnn import knn
    g = golden("knn_cases.npz")
    pts = g["ties_perm_x"]
    idx = knn(_view(pts, "perm", cuda), 20).cpu().numpy()
    pd = oracle.pairwise(_cpu_view(pts, "perm"))
    vals = np.take_along_axis(pd, idx, 2)
    assert_knn_equivalent(idx, vals, g["ties_perm_idx"], g["ties_perm_val"])


@pytest.mark.parametrize("B,C,N,k", [(1, 3, 16, 16), (2, 3, 77, 1), (2, 5, 129, 7), (3, 16, 200, 16),
                                     (2, 31, 333, 20), (1, 64, 1000, 24), (2, 100, 257, 33), (1, 128, 520, 40),
                                     (1, 3, 64, 64), (2, 12, 100, 50), (1, 9, 4096, 20)])
@pytest.mark.parametrize("layout", ["bcn", "perm"])
def test_knn_vs_oracle_ragged(cuda, B, C, N, k, layout):
    from models.dgcnn import knn
    pts = synth.relu_normal(B * 1000 + C * 10 + N, (B, N, C)) if C > 3 else synth.cube_clouds(B, N, N + k)
    idx = knn(_view(pts, layout, cuda), k).cpu().numpy()
    ref_idx, ref_vals = oracle.knn(_cpu_view(pts, layout), k, return_values=True)
    pd = oracle.pairwise(_cpu_view(pts, layout)) if N <= 1024 else None
    if pd is not None:
        assert_knn_equivalent(idx, np.take_along_axis(pd, idx, 2), ref_idx, ref_vals)
    else:
        np.testing.assert_array_equal(idx, ref_idx)


def test_knn_full_size_hashes(cuda):
    """Size-independent parity at BASELINE.json's full sizes: the selected
    distance values hash equal to the reference's, indices equal the oracle's."""
    from models.dgcnn import knn
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        H = json.load(f)
    gens = {"cfg2_layer1": lambda: synth.cube_clouds(32, 1024, 0),
            "cfg3_layer1": lambda: synth.cube_clouds(32, 2048, 0),
            "cfg5_layer1": lambda: synth.s3dis_blocks(24, 4096, 2),
            "ties_layer1": lambda: synth.tie_clouds(32, 1024, 1)}
    for name, gen in gens.items():
        h = H[name]
        pts = gen()
        idx = knn(_view(pts, "perm", cuda), h["k"]).cpu().numpy()
        ref_idx, ref_vals = oracle.knn(_cpu_view(pts, "perm"), h["k"], return_values=True)
        np.testing.assert_array_equal(idx, ref_idx)   # canonical order is deterministic
        assert hashlib.sha256(ref_vals.tobytes()).hexdigest() == h["val_sha256"], name
        if not h["boundary_ties"]:
            assert hashlib.sha256(idx.astype(np.int32).tobytes()).hexdigest() == h["idx_sha256"], name


@pytest.mark.parametrize("B", [4, 16])
def test_knn_feature_space_sizes(cuda, B):
    """Feature-space kNN shapes of DGCNN blocks 2-4 (C=64/128, contiguous) at cfg2 N;
    4 clouds keep one query group per wave at C = 128 (knn_small), 16 take two."""
    from models.dgcnn import knn
    for C in (64, 128):
        pts = synth.relu_normal(3 + C + B, (B, 1024, C))
        idx = knn(_view(pts, "bcn", cuda), 20).cpu().numpy()
        np.testing.assert_array_equal(idx, oracle.knn(_cpu_view(pts, "bcn"), 20))


def test_knn_errors(cuda):
    from models.dgcnn import knn
    x = torch.zeros(1, 3, 8, device=cuda)
    with pytest.raises(RuntimeError):
        knn(x, 9)
    # a host tensor takes the CPU path (dgx.cpu) and gives the device's answer
    pts = synth.cube_clouds(2, 300, 9)
    host = knn(torch.from_numpy(pts).permute(0, 2, 1), 12)
    dev = knn(torch.from_numpy(pts).to(cuda).permute(0, 2, 1), 12)
    assert host.device.type == "cpu" and torch.equal(host, dev.cpu())


def _lane_clustered(N, C, seed):
    """Points whose index has (j >> 2) & 3 == 0 sit in a tight cluster, the rest
    far away: every cluster query's true top-k lies in ONE of the kernel's four
    per-lane candidate quarters, which overflows the per-lane lists and forces
    the exact fix-up pass (knn_fix_kernel)."""
    pts = synth.uniform(seed, (1, N, C)).astype(np.float32) * 100.0 + 50.0
    near = ((np.arange(N) >> 2) & 3) == 0
    pts[0, near] = synth.uniform(seed + 1, (int(near.sum()), C)).astype(np.float32) * 1e-2
    return pts


@pytest.mark.parametrize("C,N,k", [(3, 256, 20), (3, 1024, 40), (64, 512, 20), (128, 300, 64), (9, 2048, 16)])
def test_knn_list_overflow_fixup(cuda, C, N, k):
    from dgx.ops import knn_raw
    pts = _lane_clustered(N, C, C + N)
    for layout in ("bcn", "perm"):
        idx, vals = knn_raw(_view(pts, layout, cuda), k, return_values=True)
        ref_idx, ref_vals = oracle.knn(_cpu_view(pts, layout), k, return_values=True)
        np.testing.assert_array_equal(idx.cpu().numpy(), ref_idx)
        np.testing.assert_array_equal(vals.cpu().numpy(), ref_vals)


@pytest.mark.parametrize("N", [300, 2048])
def test_knn_all_points_equal(cuda, N):
    """Every distance ties: the canonical answer is indices 0..k-1 for every row
    (N = 2048: more than FIX_CAP candidates reach T0, the arg-max path)."""
    from models.dgcnn import knn
    pts = np.full((2, N, 3), 0.25, np.float32)
    idx = knn(_view(pts, "perm", cuda), 20).cpu().numpy()
    np.testing.assert_array_equal(idx, oracle.knn(_cpu_view(pts, "perm"), 20))
    np.testing.assert_array_equal(idx[0, 7], np.arange(20))


@pytest.mark.parametrize("B,C,N", [(2, 3, 77), (1, 9, 1000), (2, 64, 1024), (1, 100, 257), (1, 128, 520)])
@pytest.mark.parametrize("layout", ["bcn", "perm"])
def test_knn_prepare_norms_match_sqnorm(cuda, B, C, N, layout):
    """dgx_knn_prepare_f32's fused |x|^2 is bit-identical to dgx_sqnorm_f32 (and
    to the oracle's restatement of the reference's reduction order)."""
    from dgx import _native as nat
    from dgx.ops import reduction_order
    pts = synth.relu_normal(B * 7 + C + N, (B, N, C))
    x = _view(pts, layout, cuda)
    L = nat.lib()
    sB, sC, sN = x.stride()
    order = reduction_order(x)
    xx0 = torch.empty(B * N, dtype=torch.float32, device=cuda)
    xx1 = torch.full((B * N,), float("nan"), dtype=torch.float32, device=cuda)
    nb = L.dgx_knn_image_bytes(B, C, N)
    img = torch.empty((nb + 3) // 4, dtype=torch.float32, device=cuda)
    s = nat.stream_of(x)
    nat.check(L.dgx_sqnorm_f32(nat.ptr(x), sB, sC, sN, B, C, N, order, nat.ptr(xx0), s), "sqnorm")
    nat.check(L.dgx_knn_prepare_f32(nat.ptr(x), sB, sC, sN, B, C, N, order, nat.ptr(xx1), nat.ptr(img), nb, s),
              "prepare")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(xx0.cpu().numpy().view(np.uint32), xx1.cpu().numpy().view(np.uint32))
    ref = oracle.sqnorm(_cpu_view(pts, layout)).reshape(-1)
    np.testing.assert_array_equal(xx1.cpu().numpy().view(np.uint32), ref.astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("B,N,k,layout", [(3, 1024, 20, "perm"), (2, 2048, 40, "bcn"), (1, 4096, 64, "perm"),
                                          (2, 256, 16, "bcn"), (2, 777, 33, "perm")])
def test_knn_coordinate_clouds_duplicates_and_flat(cuda, B, N, k, layout):
    """Coordinate clouds (reference dgcnn.py:6-12 on xyz input) with duplicated
    points (exact distance ties, some at the k-th value) and a degenerate flat
    cloud (one coordinate constant): selected values bit-exact, indices in
    canonical order, against the oracle."""
    from dgx.ops import knn_raw
    pts = synth.cube_clouds(B, N, N + k)
    pts[:, N // 2:N // 2 + N // 8] = pts[:, :N // 8]            # duplicated points: ties
    if B > 1:
        pts[1, :, 2] = 0.0                                      # a flat cloud (one empty grid axis)
    f = torch.from_numpy(pts).permute(0, 2, 1)
    if layout == "bcn":
        f = f.contiguous()
    x = f.to(cuda)
    idx, vals = oracle.knn(f, k, return_values=True)
    got_idx, got_vals = knn_raw(x, k, return_values=True)
    assert_knn_equivalent(got_idx.cpu().numpy(), got_vals.cpu().numpy(), idx, vals)


@pytest.mark.parametrize("B,N,Co", [(4, 1024, 64), (2, 2048, 128), (3, 96, 64)])
def test_apply_writes_next_knn_image(cuda, B, N, Co):
    """dgx_bn_lrelu_apply_knn_image_f32 (EdgeConv apply + the next block's kNN
    operands) equals dgx_bn_lrelu_apply_f32 followed by dgx_knn_prepare_f32 on
    the written concat slice, bit for bit (|x|^2 in the reference's strided
    order), and the kNN from the prepared buffers equals the plain kNN."""
    from dgx import _native as nat
    from dgx.ops import knn_image_buffers, knn_raw
    L = nat.lib()
    g = torch.Generator().manual_seed(N + Co)
    M, total, off = B * N, Co + 32, 16
    ysel = torch.randn(M, Co, generator=g).to(cuda)
    scale, shift = torch.randn(Co, generator=g).to(cuda), torch.randn(Co, generator=g).to(cuda)
    outs = []
    for fused in (False, True):
        xcat = torch.zeros(M, total, device=cuda)
        x16 = torch.zeros(M, total, dtype=torch.bfloat16, device=cuda)
        out, out16 = xcat[:, off:off + Co], x16[:, off:off + Co]
        xx, img = knn_image_buffers(B, Co, N, cuda)
        st = nat.stream_of(ysel)
        if fused:
            nat.check(L.dgx_bn_lrelu_apply_knn_image_f32(nat.f32(ysel), B, N, Co, nat.f32(scale), nat.f32(shift), 0.2,
                                                         nat.f32(out), total, nat.ptr(out16), nat.f32(xx),
                                                         nat.f32(img), img.numel() * 4, st), "fused")
        else:
            nat.check(L.dgx_bn_lrelu_apply_f32(nat.f32(ysel), M, Co, nat.f32(scale), nat.f32(shift), 0.2,
                                               nat.f32(out), total, nat.ptr(out16), st), "apply")
            nat.check(L.dgx_knn_prepare_f32(nat.f32(xcat[:, off:]), N * total, 1, total, B, Co, N, nat.ORDER_STRIDED,
                                            nat.f32(xx), nat.f32(img), img.numel() * 4, st), "prepare")
        outs.append((xcat, x16, xx, img))
    for a, b in zip(*outs):
        assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32),
                           b.view(torch.int16) if b.dtype == torch.bfloat16 else b.view(torch.int32))
    xcat, _, xx, img = outs[1]
    kw = dict(order=nat.ORDER_STRIDED, out_dtype=torch.int32, strides=(N * total, 1, total), shape=(B, Co, N))
    a = knn_raw(xcat[:, off:], 20, prepared=(xx, img), **kw)
    b = knn_raw(xcat[:, off:], 20, **kw)
    assert torch.equal(a, b)
