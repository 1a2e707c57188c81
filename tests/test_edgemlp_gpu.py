"""a6 parity: PositionEmbedding's fused per-edge MLP (dgx.edgemlp, csrc/edgemlp.hip)
against the reference op sequence (models/layers.py:45-52: get_graph_feature ->
conv1 -> conv2 -> max over k) recomputed in fp64 on the CPU from the same
neighbour sets (the engine's kNN is bit-exact with the reference, tested in
test_knn_gpu.py)."""
import numpy as np
import pytest
import torch

import oracle
from conftest import rel_err
from oracle import reference as R

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _convs(seed, cin2=6, c1=64, c2=128, neg=True):
    g = torch.Generator().manual_seed(seed)

    def block(ci, co):
        blk = torch.nn.Sequential(torch.nn.Conv2d(ci, co, 1, bias=False), torch.nn.BatchNorm2d(co),
                                  torch.nn.LeakyReLU(0.2))
        with torch.no_grad():
            blk[0].weight.copy_(torch.randn(co, ci, 1, 1, generator=g) / np.sqrt(ci))
            gam = 1.0 + 0.3 * torch.randn(co, generator=g)
            if neg:
                gam[::5] *= -1.0  # decreasing BN affine on some channels: min-over-k path
            blk[1].weight.copy_(gam)
            blk[1].bias.copy_(0.2 * torch.randn(co, generator=g))
        return blk
    return block(cin2, c1), block(c1, c2)


def _reference(x64, idx, conv1, conv2):
    e = R.graph_feature(x64, idx.shape[-1], idx=idx)
    return conv2(conv1(e)).max(dim=-1)[0]


def _frac_close(a, b, tol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float((np.abs(a - b) <= tol * max(np.abs(b).max(), 1e-30)).mean())


@pytest.mark.parametrize("B,N,k", [(2, 256, 20), (1, 500, 40), (3, 128, 7)])
def test_edge_mlp_train_matches_reference(cuda, B, N, k):
    from dgx import synth
    from dgx.edgemlp import edge_mlp2
    conv1, conv2 = _convs(11 + k)
    ref1, ref2 = _convs(11 + k)
    ref1, ref2 = ref1.double().train(), ref2.double().train()
    conv1, conv2 = conv1.to(cuda).train(), conv2.to(cuda).train()
    pts = synth.cube_clouds(B, N, 40 + N)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1).requires_grad_(True)
    y = edge_mlp2(x, k, conv1, conv2, True)
    assert y.shape == (B, 128, N)
    gout = torch.from_numpy(synth.uniform(9, (B, 128, N)) - 0.5).float()
    y.backward(gout.to(cuda))

    x64 = torch.from_numpy(pts).double().permute(0, 2, 1).requires_grad_(True)
    idx = oracle.knn(torch.from_numpy(pts).permute(0, 2, 1), k)
    ref = _reference(x64, torch.as_tensor(idx).long(), ref1, ref2)
    ref.backward(gout.double())

    assert rel_err(y.detach().cpu(), ref.detach()) < TOL
    # running statistics of both BatchNorms (momentum update, unbiased var)
    for got, want in ((conv1[1], ref1[1]), (conv2[1], ref2[1])):
        assert rel_err(got.running_mean.cpu(), want.running_mean) < 1e-4
        assert rel_err(got.running_var.cpu(), want.running_var) < 1e-4
        assert int(got.num_batches_tracked) == 1
    # gradients: a LeakyReLU kink or near-tie max that fp32 rounding flips moves a
    # handful of elements; everything else must agree to 1e-3 of the tensor's scale
    pairs = [(x.grad, x64.grad)]
    for got, want in ((conv1, ref1), (conv2, ref2)):
        pairs += [(got[0].weight.grad, want[0].weight.grad), (got[1].weight.grad, want[1].weight.grad),
                  (got[1].bias.grad, want[1].bias.grad)]
    for got, want in pairs:
        g, w = got.cpu().double(), want.detach()
        assert rel_err(g, w) < 1e-2 and _frac_close(g, w, TOL) >= 0.99, (rel_err(g, w), _frac_close(g, w, TOL))


def test_edge_mlp_eval_matches_reference(cuda):
    from dgx import synth
    from dgx.edgemlp import edge_mlp2
    B, N, k = 2, 300, 16
    conv1, conv2 = _convs(5)
    ref1, ref2 = _convs(5)
    for blk in (conv1, conv2, ref1, ref2):
        with torch.no_grad():
            blk[1].running_mean.copy_(torch.linspace(-0.3, 0.3, blk[1].running_mean.numel()))
            blk[1].running_var.copy_(torch.linspace(0.5, 2.0, blk[1].running_var.numel()))
    ref1, ref2 = ref1.double().eval(), ref2.double().eval()
    conv1, conv2 = conv1.to(cuda).eval(), conv2.to(cuda).eval()
    pts = synth.cube_clouds(B, N, 3)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
    with torch.no_grad():
        y = edge_mlp2(x, k, conv1, conv2, False)
        idx = oracle.knn(torch.from_numpy(pts).permute(0, 2, 1), k)
        ref = _reference(torch.from_numpy(pts).double().permute(0, 2, 1), torch.as_tensor(idx).long(), ref1, ref2)
    assert rel_err(y.cpu(), ref) < TOL


# SURVEY §8(c)'s bf16 bar, held by the output, the input gradient and all six
# parameter gradients (max-abs normwise) against the fp64 oracle routed by the
# engine's validated decisions.
BF16_TOL = 2e-2


@pytest.mark.parametrize("mode,B,N,k,c2", [("bf16", 4, 2048, 40, 128),   # cfg4 geometry (B 32 over 8 GPUs)
                                           ("bf16", 2, 512, 20, 128), ("bf16", 2, 1024, 40, 128),
                                           ("bf16", 3, 256, 10, 64), ("bf16", 1, 300, 33, 64),
                                           ("fp32", 4, 2048, 40, 128), ("fp32", 3, 128, 7, 128)])
def test_edge_mlp_routed(cuda, mode, B, N, k, c2):
    """PositionEmbedding's edge stage (layers.py:45-52) against the fp64 oracle
    routed by the engine's own decisions (oracle.reference.edge_mlp2_routed):
    the kNN graph equals the oracle's, every conv2 max slot / LeakyReLU sign is
    validated by an fp64 recomputation in the engine's arithmetic
    (conftest.edge_mlp_decisions), then output, dx and the gradients of both
    convs' weights and BN affines are held to BF16_TOL (bf16 mode: the fused
    forward/backward kernels bench.py times) or TOL (fp32 parity mode).
    k = 40/20/10/33/7 cover 3, 2, 1 and partial 16-row tiles per point;
    C2 = 64 is the semseg width (fused forward, unfused backward)."""
    import dgx.edgeconv as E
    from dgx import precision, synth
    from dgx.edgemlp import edge_mlp2
    from conftest import edge_mlp_decisions
    conv1, conv2 = _convs(31 + k, c2=c2)
    init = {f"c{i}.{n}": t.detach().clone() for i, blk in ((1, conv1), (2, conv2)) for n, t in blk.state_dict().items()}
    conv1, conv2 = conv1.to(cuda).train(), conv2.to(cuda).train()
    pts = synth.cube_clouds(B, N, 50 + N + k)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1).requires_grad_(True)
    gout = torch.from_numpy(synth.uniform(51 + k, (B, c2, N)) - 0.5).float()
    precision.set(mode)
    E.set_debug_capture({})
    try:
        y = edge_mlp2(x, k, conv1, conv2, True)
        y.backward(gout.to(cuda))
        cap = E.debug_capture()
    finally:
        E.set_debug_capture(None)
        precision.set("fp32")
    idx = cap["emlp"]["idx"].view(B, N, k)
    np.testing.assert_array_equal(idx.long().cpu().numpy(), oracle.knn(torch.from_numpy(pts).permute(0, 2, 1), k))
    zpos1, arg2, zpos2, dec = edge_mlp_decisions(cap, B, N, k, conv2[0].weight)
    p64 = {n: t.to(cuda).double() for n, t in init.items() if not n.endswith("num_batches_tracked")}
    for n in ("c1.0.weight", "c1.1.weight", "c1.1.bias", "c2.0.weight", "c2.1.weight", "c2.1.bias"):
        p64[n].requires_grad_(True)
    x64 = torch.from_numpy(pts).to(cuda).double().permute(0, 2, 1).requires_grad_(True)
    bns = [{n: p64[f"c{i}.1.{n}"] for n in ("weight", "bias", "running_mean", "running_var")} for i in (1, 2)]
    ref, _ = R.edge_mlp2_routed(x64, p64["c1.0.weight"], bns[0], p64["c2.0.weight"], bns[1], idx.long(), zpos1,
                                arg2, zpos2)
    ref.backward(gout.to(cuda).double())
    tol = BF16_TOL if mode == "bf16" else TOL
    errs = {"out": rel_err(y.detach().cpu(), ref.detach().cpu()), "x": rel_err(x.grad.cpu(), x64.grad.cpu())}
    for i, blk in ((1, conv1), (2, conv2)):
        for n, t in (("0.weight", blk[0].weight), ("1.weight", blk[1].weight), ("1.bias", blk[1].bias)):
            errs[f"c{i}.{n}"] = rel_err(t.grad.cpu(), p64[f"c{i}.{n}"].grad.cpu())
    print(f"{mode} B{B} N{N} k{k} C2 {c2}: decisions (gap, flip) {dec}; rel err",
          {n: f"{e:.2e}" for n, e in errs.items()})
    for n, e in errs.items():
        assert e < tol, (n, e, tol)
    for i, blk in ((1, conv1), (2, conv2)):   # running statistics (momentum update, unbiased var)
        for n in ("running_mean", "running_var"):
            assert rel_err(getattr(blk[1], n).cpu(), bns[i - 1][n].cpu()) < (tol if mode == "bf16" else 1e-4), (i, n)


def test_edge_mlp_bf16_kernels_equal_fp32_kernels(cuda):
    """The bf16 variants of the edge-MLP kernels compute exactly what the fp32
    variants compute, rounded once (RNE) where they store: with the fp32 mode's
    1e-3 parity above, the bf16 mode differs from it only by operand rounding."""
    from dgx import _native as nat
    from dgx.ops import knn_raw, reduction_order
    L = nat.lib()
    B, N, k, C1, C2 = 2, 200, 12, 64, 128
    M, E = B * N, B * N * k
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.rand(B, 3, N, generator=g).to(cuda)
    idx = knn_raw(x, k, order=reduction_order(x), out_dtype=torch.int32)
    PQ = torch.randn(M, 2 * C1, generator=g).to(cuda)
    sc1, sh1 = torch.randn(C1, generator=g).to(cuda), torch.randn(C1, generator=g).to(cuda)
    st = nat.stream_of(x)
    h32 = torch.empty(E, C1, device=cuda)
    h16 = torch.empty(E, C1, device=cuda, dtype=torch.bfloat16)
    for out, flag in ((h32, 0), (h16, 1)):
        nat.check(L.dgx_edge_mlp_h1_f32(nat.ptr(PQ), 2 * C1, nat.ptr(idx), B, N, k, C1, nat.ptr(sc1), nat.ptr(sh1),
                                        0.2, nat.ptr(out), flag, st), "h1")
    assert torch.equal(h32.to(torch.bfloat16), h16)
    # the fp32 h1 itself: LReLU(a (P_j + Q_i) + b) on the engine's neighbour sets
    il = idx.long().view(M, k) + (torch.arange(M, device=cuda) // N * N).view(M, 1)
    y = PQ[il.reshape(-1), :C1] + PQ[:, C1:].repeat_interleave(k, dim=0)
    z = torch.addcmul(sh1, sc1, y)
    assert rel_err(h32.cpu(), torch.where(z > 0, z, 0.2 * z).cpu()) < 1e-6
    # max over k: bf16 Z vs the same values in fp32 -> identical selection
    z16 = torch.randn(E, C2, generator=g).to(cuda).to(torch.bfloat16)
    sc2 = torch.randn(C2, generator=g).to(cuda)
    sel = [torch.empty(M, C2, device=cuda) for _ in range(2)]
    arg = [torch.empty(M, C2, device=cuda, dtype=torch.uint8) for _ in range(2)]
    for i, (zz, flag) in enumerate(((z16.float().contiguous(), 0), (z16, 1))):
        nat.check(L.dgx_edge_mlp_max_f32(nat.ptr(zz), flag, B, N, k, C2, nat.ptr(sc2), nat.ptr(sel[i]),
                                         nat.ptr(arg[i]), st), "max")
    assert torch.equal(sel[0], sel[1]) and torch.equal(arg[0], arg[1])
    zf = z16.float().view(M, k, C2)
    want = torch.where(sc2 < 0, zf.min(dim=1)[0], zf.max(dim=1)[0])
    assert torch.equal(sel[0], want)
    assert torch.equal(torch.gather(zf, 1, arg[0].long().unsqueeze(1)).squeeze(1), want)
    # dense BN2 backward: bf16 in/out == fp32 in/out rounded
    dzv = torch.randn(M, C2, generator=g).to(cuda)
    sarg = torch.randint(0, k, (M, C2), generator=g).to(cuda).to(torch.uint8)
    c0, c1 = torch.randn(C2, generator=g).to(cuda), torch.randn(C2, generator=g).to(cuda)
    d32 = torch.empty(E, C2, device=cuda)
    d16 = torch.empty(E, C2, device=cuda, dtype=torch.bfloat16)
    for zz, out, flag in ((z16.float().contiguous(), d32, 0), (z16, d16, 1)):
        nat.check(L.dgx_edge_mlp_dz_f32(nat.ptr(dzv), nat.ptr(sarg), nat.ptr(zz), flag, B, N, k, C2, nat.ptr(sc2),
                                        nat.ptr(c0), nat.ptr(c1), nat.ptr(out), st), "dz2")
    assert torch.equal(d32.to(torch.bfloat16), d16)
    hit = sarg.long().unsqueeze(1) == torch.arange(k, device=cuda).view(1, k, 1)
    ref = torch.addcmul(c0, c1, zf) + torch.where(hit, sc2 * dzv.unsqueeze(1), torch.zeros((), device=cuda))
    assert rel_err(d32.view(M, k, C2).cpu(), ref.cpu()) < 1e-6


def test_edge_mlp_mixed_devices_and_bad_shapes(cuda):
    from dgx.edgemlp import edge_mlp2
    conv1, conv2 = _convs(1)
    conv1, conv2 = conv1.to(cuda), conv2.to(cuda)
    with pytest.raises(RuntimeError):
        edge_mlp2(torch.rand(1, 3, 64), 8, conv1, conv2, True)  # host cloud, device weights
    with pytest.raises(RuntimeError):
        edge_mlp2(torch.zeros(1, 4, 64, device=cuda), 8, conv1, conv2, True)  # conv1 expects 2*3 channels
