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


def test_knn_feature_space_sizes(cuda):
    """Feature-space kNN shapes of DGCNN blocks 2-4 (C=64/128, contiguous) at cfg2 N."""
    from models.dgcnn import knn
    for C in (64, 128):
        pts = synth.relu_normal(3 + C, (4, 1024, C))
        idx = knn(_view(pts, "bcn", cuda), 20).cpu().numpy()
        np.testing.assert_array_equal(idx, oracle.knn(_cpu_view(pts, "bcn"), 20))


def test_knn_errors(cuda):
    from models.dgcnn import knn
    x = torch.zeros(1, 3, 8, device=cuda)
    with pytest.raises(RuntimeError):
        knn(x, 9)
    with pytest.raises(RuntimeError):
        knn(torch.zeros(1, 3, 8), 2)  # CPU tensors are not silently served


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


@pytest.mark.parametrize("C,N,k,layout", [(64, 1024, 20, "pm"), (128, 2048, 40, "pm"), (64, 777, 20, "bcn"),
                                          (3, 500, 16, "perm"), (9, 1000, 20, "bcn")])
def test_knn_seeded_equals_unseeded(cuda, C, N, k, layout):
    """Admission seeds (dgx_knn_seed_f32 + dgx_knn_select_seeded_f32) never change
    the result: seeded by the exact kNN itself (the bound equals the k-th
    value: only the top-k and its ties are admitted), by random distinct ids (a
    loose bound), by another layer's graph (what EdgeConv blocks 2-4 pass), and
    by an INVALID seed list (k copies of the query itself: the bound exceeds
    the k-th value, every row falls short of k admitted candidates and is
    recomputed exactly by the fix-up) — all bit-identical to the unseeded kNN
    and to the oracle."""
    import oracle
    from dgx import synth
    from dgx.ops import knn_raw
    B = 2
    if C == 3:
        f = torch.from_numpy(synth.cube_clouds(B, N, 5)).permute(0, 2, 1)
    else:
        f = torch.from_numpy(synth.relu_normal(6 + C, (B, C, N)))
    if layout == "pm":   # point-major memory, as the engine's concat buffer
        f = f.permute(0, 2, 1).contiguous().permute(0, 2, 1)
    elif layout == "perm":
        f = f.permute(0, 2, 1).contiguous().permute(0, 2, 1)
    x = f.to(cuda)
    base = knn_raw(x, k, out_dtype=torch.int32)
    np.testing.assert_array_equal(base.cpu().numpy(), oracle.knn(f, k))
    g = torch.Generator().manual_seed(C + N)
    rnd = torch.argsort(torch.rand(B, N, N, generator=g), dim=-1)[..., :k + 3].to(torch.int32)
    other = knn_raw((x * x).contiguous(), k, out_dtype=torch.int32)        # a different graph of the same points
    selfs = torch.arange(N, dtype=torch.int32).view(1, N, 1).expand(B, N, k).contiguous()
    for name, seeds in (("exact", base), ("random", rnd), ("other graph", other), ("invalid", selfs)):
        got = knn_raw(x, k, out_dtype=torch.int32, seeds=seeds.to(cuda).contiguous())
        assert torch.equal(got, base), name


@pytest.mark.parametrize("B,N,k,layout", [(3, 1024, 20, "perm"), (2, 2048, 40, "bcn"), (1, 4096, 64, "perm"),
                                          (2, 256, 16, "bcn"), (2, 777, 33, "perm")])
def test_knn_spatial_seeds_change_nothing(cuda, monkeypatch, B, N, k, layout):
    """Coordinate clouds take spatial admission seeds (dgx_knn_spatial_seed_f32):
    the result is bit-identical to the unseeded selection and to the oracle,
    including clouds of duplicated points (exact ties at the seed) and a
    degenerate flat cloud."""
    import oracle
    from dgx import ops, synth
    from dgx.ops import knn_raw
    pts = synth.cube_clouds(B, N, N + k)
    pts[:, N // 2:N // 2 + N // 8] = pts[:, :N // 8]            # duplicated points: ties
    if B > 1:
        pts[1, :, 2] = 0.0                                      # a flat cloud (one empty grid axis)
    f = torch.from_numpy(pts).permute(0, 2, 1)
    if layout == "bcn":
        f = f.contiguous()
    x = f.to(cuda)
    monkeypatch.setattr(ops, "SPATIAL_SEEDS", True)
    seeded = knn_raw(x, k)
    monkeypatch.setattr(ops, "SPATIAL_SEEDS", False)
    plain = knn_raw(x, k)
    assert torch.equal(seeded, plain)
    idx, vals = oracle.knn(f, k, return_values=True)
    got_idx, got_vals = knn_raw(x, k, return_values=True)
    from conftest import assert_knn_equivalent
    assert_knn_equivalent(seeded.cpu().numpy(), got_vals.cpu().numpy(), idx, vals)


@pytest.fixture
def knn3_variant():
    from dgx import _native as nat
    nat.lib().dgx_knn_set_variant(1)
    yield
    nat.lib().dgx_knn_set_variant(0)


@pytest.mark.parametrize("B,N,k,layout", [(2, 77, 1, "perm"), (1, 64, 64, "bcn"), (3, 1024, 20, "perm"),
                                          (2, 2048, 40, "bcn"), (1, 4096, 20, "perm"), (2, 333, 33, "bcn")])
def test_knn3_variant_vs_oracle(cuda, knn3_variant, B, N, k, layout):
    """The VALU 3-channel selection kernel (dgx_knn_set_variant(1), off by
    default: measured no faster) returns the reference's neighbours too."""
    from models.dgcnn import knn
    pts = synth.cube_clouds(B, N, 3 * N + k)
    idx = knn(_view(pts, layout, cuda), k).cpu().numpy()
    ref_idx, ref_vals = oracle.knn(_cpu_view(pts, layout), k, return_values=True)
    if N <= 1024:
        pd = oracle.pairwise(_cpu_view(pts, layout))
        assert_knn_equivalent(idx, np.take_along_axis(pd, idx, 2), ref_idx, ref_vals)
    else:
        np.testing.assert_array_equal(idx, ref_idx)


def test_knn3_variant_ties(golden, cuda, knn3_variant):
    from models.dgcnn import knn
    g = golden("knn_cases.npz")
    pts = g["ties_perm_x"]
    idx = knn(_view(pts, "perm", cuda), 20).cpu().numpy()
    pd = oracle.pairwise(_cpu_view(pts, "perm"))
    assert_knn_equivalent(idx, np.take_along_axis(pd, idx, 2), g["ties_perm_idx"], g["ties_perm_val"])


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


@pytest.mark.parametrize("B,N,Co,layout", [(32, 1024, 64, "perm"), (3, 777, 24, "bcn"), (2, 2048, 64, "perm")])
def test_prepare_with_block1_pq(cuda, B, N, Co, layout):
    """dgx_knn_prepare_pq_f32: the kNN operands of a coordinate cloud equal
    dgx_knn_prepare_f32's and its PQ rows equal dgx_gemm_smallk_split_f32's,
    bit for bit."""
    from dgx import _native as nat
    from dgx import gemm as G
    from dgx.ops import knn_image_buffers, reduction_order
    L = nat.lib()
    x = _view(synth.cube_clouds(B, N, N + Co), layout, cuda)
    w = torch.randn(Co, 6, 1, 1, generator=torch.Generator().manual_seed(Co)).to(cuda)
    order = reduction_order(x)
    st = nat.stream_of(x)
    xx1, img1 = knn_image_buffers(B, 3, N, cuda)
    xx2, img2 = knn_image_buffers(B, 3, N, cuda)
    pq = torch.empty(B * N, 2 * Co, device=cuda)
    nat.check(L.dgx_knn_prepare_f32(nat.f32(x), *x.stride(), B, 3, N, order, nat.f32(xx1), nat.f32(img1),
                                    img1.numel() * 4, st), "prepare")
    nat.check(L.dgx_knn_prepare_pq_f32(nat.f32(x), *x.stride(), B, 3, N, order, nat.f32(xx2), nat.f32(img2),
                                       img2.numel() * 4, nat.f32(w), Co, nat.f32(pq), 2 * Co, st), "prepare pq")
    ref = G.mm_smallk_split(x.permute(0, 2, 1).reshape(B * N, 3), w, Co)
    assert torch.equal(xx1, xx2) and torch.equal(img1, img2)
    assert torch.equal(pq.view(torch.int32), ref.view(torch.int32))
