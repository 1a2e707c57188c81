"""a3/a5/a8 parity: fused EdgeConv chain and DGCNN vs the reference's goldens
(1e-3 relative fp32)."""
import copy
import types

import numpy as np
import pytest
import torch

import oracle
from conftest import check_decisions, rel_err, validate_dgcnn_decisions
from oracle import reference as R

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _block(w, gamma, beta, dev):
    co, c2 = w.shape[0], w.shape[1]
    blk = torch.nn.Sequential(torch.nn.Conv2d(c2, co, 1, bias=False), torch.nn.BatchNorm2d(co),
                              torch.nn.LeakyReLU(0.2, inplace=True)).to(dev)
    with torch.no_grad():
        blk[0].weight.copy_(torch.from_numpy(w))
        blk[1].weight.copy_(torch.from_numpy(gamma))
        blk[1].bias.copy_(torch.from_numpy(beta))
    return blk


def frac_close(a, b, tol=TOL):
    """fraction of elements with |a-b| <= tol * max|b| (gradient goldens: a
    LeakyReLU kink or max near-tie that fp32 reordering flips moves a handful of
    elements; everything else must agree to tol)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float((np.abs(a - b) <= tol * max(np.abs(b).max(), 1e-30)).mean())


class Capture:
    """Record the engine's routing decisions (per block: idx, arg, zpos)."""

    def __enter__(self):
        import dgx.edgeconv as E
        self.E = E
        E.set_debug_capture({})
        return E.debug_capture()

    def __exit__(self, *exc):
        self.E.set_debug_capture(None)


def test_edgeconv_block_golden(golden, cuda):
    from dgx.edgeconv import edgeconv_stack
    g = golden("edgeconv_block.npz")
    k = int(g["k"])
    blk = _block(g["weight"], g["gamma"], g["beta"], cuda)
    x = torch.from_numpy(g["x"]).to(cuda).requires_grad_(True)
    B, C, N = x.shape
    out = edgeconv_stack(x, k, [blk], True)                       # (B*N, Co) point-major
    y = out.view(B, N, -1).permute(0, 2, 1)
    assert rel_err(y.detach().cpu(), g["out"]) < TOL
    y.backward(torch.from_numpy(g["gout"]).to(cuda))
    for got, key in ((x.grad, "dx"), (blk[0].weight.grad, "dweight"), (blk[1].weight.grad, "dgamma"),
                     (blk[1].bias.grad, "dbeta")):
        assert frac_close(got.cpu(), g[key]) >= 0.99, key
    assert rel_err(blk[1].running_mean.cpu(), g["running_mean"]) < 1e-5
    assert rel_err(blk[1].running_var.cpu(), g["running_var"]) < 1e-5
    assert int(blk[1].num_batches_tracked) == 1


@pytest.mark.parametrize("C,Co,N,k", [(3, 64, 300, 20), (64, 128, 256, 16), (128, 256, 130, 10), (64, 64, 1024, 20),
                                      (9, 64, 4096, 20)])   # cfg5 block 1: S3DIS 9-channel input, N 4096
def test_edgeconv_block_routed(cuda, C, Co, N, k):
    """Strict 1e-3 parity of outputs AND all gradients against the fp64 oracle
    that follows the engine's routing decisions (ragged N, negative gammas)."""
    from dgx.edgeconv import edgeconv_stack
    torch.manual_seed(C + Co + N)
    B = 2
    x = torch.randn(B, C, N)
    w = (torch.randn(Co, 2 * C, 1, 1) / (2 * C) ** 0.5).numpy()
    gamma, beta = torch.randn(Co).numpy(), (0.1 * torch.randn(Co)).numpy()
    blk = _block(w, gamma, beta, cuda)
    xg = x.to(cuda).requires_grad_(True)
    with Capture() as cap:
        out = edgeconv_stack(xg, k, [blk], True).view(B, N, Co).permute(0, 2, 1)
    gout = torch.randn(B, Co, N)
    out.backward(gout.to(cuda))
    idx, arg, zpos = cap[("fwd", 0)]
    xc = x.double().requires_grad_(True)
    wc = torch.from_numpy(w).double().requires_grad_(True)
    gc = torch.from_numpy(gamma).double().requires_grad_(True)
    bc = torch.from_numpy(beta).double().requires_grad_(True)
    bn = {"weight": gc, "bias": bc, "running_mean": torch.zeros(Co, dtype=torch.float64),
          "running_var": torch.ones(Co, dtype=torch.float64)}
    ref, z64 = R.edgeconv_block_routed(xc, wc, bn, idx.cpu().long(), arg.cpu(), zpos.cpu())
    check_decisions(z64, arg, zpos, B, N)
    ref.backward(gout.double())
    assert rel_err(out.detach().cpu(), ref.detach()) < TOL
    assert rel_err(xg.grad.cpu(), xc.grad) < TOL
    assert rel_err(blk[0].weight.grad.cpu(), wc.grad) < TOL
    assert rel_err(blk[1].weight.grad.cpu(), gc.grad) < TOL
    assert rel_err(blk[1].bias.grad.cpu(), bc.grad) < TOL
    assert rel_err(blk[1].running_mean.cpu(), bn["running_mean"]) < 1e-5
    assert rel_err(blk[1].running_var.cpu(), bn["running_var"]) < 1e-5


def _dgcnn_from_golden(g, dev, emb=64, k=10):
    from models.dgcnn import DGCNN
    m = DGCNN(types.SimpleNamespace(emb_dim=emb, k=k))
    m.load_state_dict({n[5:]: torch.from_numpy(g[n]) for n in g.files if n.startswith("init.")})
    return m.to(dev)


def test_dgcnn_train_golden(golden, cuda):
    g = golden("dgcnn_small.npz")
    m = _dgcnn_from_golden(g, cuda)
    m.train()
    x = torch.from_numpy(g["x"]).to(cuda)
    y = m(x)
    assert tuple(y.shape) == g["out"].shape
    assert rel_err(y.detach().cpu(), g["out"]) < TOL
    y.backward(torch.from_numpy(g["gout"]).to(cuda))
    # Unrouted gradients vs the reference's fp32 run: this fixture contains one
    # block-4 element whose BN output sits at |z| ~ 1e-7, so fp32 reordering
    # flips its LeakyReLU slope and the change propagates to every lower block
    # (found by comparing each block's routed decisions with the fixture's;
    # validate_dgcnn_decisions in conftest.py does that check). Strict 1e-3 gradient parity is
    # asserted with identical routing in test_dgcnn_train_routed.
    for n, p in m.named_parameters():
        assert rel_err(p.grad.cpu(), g["grad." + n]) < 5e-2, n
    for n, b in m.state_dict().items():
        if "running" in n:
            assert rel_err(b.cpu(), g["after." + n]) < 1e-4, n


# Gradient bar of the routed parity test: every parameter of every geometry.
# Measured engine errors are <= 1e-5 against the fp64 routed oracle (printed by
# the test; the same routed computation in torch fp32 lands at 1e-6..3e-6), so
# the bar is held 10x tighter than the 1e-3 contract.
ROUTED_GRAD_TOL = 1e-4


def _clouds(B, N, in_dims, seed):
    """(B, N, in_dims) synthetic input: unit-cube xyz clouds, or the S3DIS
    9-channel block layout (prepare_data/indoor3d_util.py:251-260) for cfg5."""
    from dgx import synth
    if in_dims == 9:
        return synth.s3dis_blocks(B, N, seed=seed)
    return synth.cube_clouds(B, N, seed)


@pytest.mark.parametrize("emb,N,k,B,in_dims", [(64, 128, 10, 2, 3), (1024, 1024, 20, 4, 3),
                                               (256, 2048, 40, 2, 3),     # cfg3 geometry (N 2048, k 40)
                                               (128, 4096, 20, 1, 3),     # cfg5 cloud size, xyz input
                                               (1024, 4096, 20, 2, 9)])   # cfg5: DGCNN(in_dims=9), S3DIS blocks
def test_dgcnn_train_routed(golden, cuda, emb, N, k, B, in_dims):
    """Strict parity of DGCNN train-mode output and EVERY parameter gradient vs
    the fp64 oracle following the engine's routing decisions, at the cfg2 /
    cfg3 / cfg5 cloud sizes (the kernels' LDS slicing changes with N) and the
    cfg5 model itself (9-channel S3DIS input, reference models/dgcnn.py:84-98
    with conv1 = Conv2d(18, 64)); one fixed bar for every gradient
    (ROUTED_GRAD_TOL)."""
    from models.dgcnn import DGCNN
    from dgx import synth
    torch.manual_seed(emb + N + (in_dims if in_dims != 3 else 0))
    m = DGCNN(types.SimpleNamespace(emb_dim=emb, k=k, in_dims=in_dims))
    init = {n: t.detach().clone() for n, t in m.state_dict().items()}
    m = m.to(cuda).train()
    pts = _clouds(B, N, in_dims, 60 + N)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
    with Capture() as cap:
        y = m(x)
    gout = torch.from_numpy(synth.uniform(61, tuple(y.shape)) - 0.5)
    y.backward(gout.to(cuda))
    decisions = [tuple(t for t in cap[("fwd", l)]) for l in range(4)]
    mask5 = y.detach() > 0
    # every block's neighbour sets and max slots / signs are the reference's own
    # (oracle kNN of the block's input, fp64 z), so routing by them is sound
    print("decision check (gap, flip):", validate_dgcnn_decisions(cap, x, k, init))

    def routed(dtype):
        params = {n: (t.to(cuda).to(dtype) if t.is_floating_point() else t.to(cuda)) for n, t in init.items()}
        for n, t in params.items():
            if t.is_floating_point() and "running" not in n:
                t.requires_grad_(True)
        dec = [(i.long(), a, z) for (i, a, z) in decisions]
        ref = R.dgcnn_routed(torch.from_numpy(pts).to(cuda).to(dtype).permute(0, 2, 1), params, dec, mask5)
        ref.backward(gout.to(cuda).to(dtype))
        return ref.detach(), params
    ref, p64 = routed(torch.float64)
    _, p32 = routed(torch.float32)
    assert rel_err(y.detach().cpu(), ref.cpu()) < TOL
    report = {}
    for n, p in m.named_parameters():
        e = rel_err(p.grad.cpu(), p64[n].grad.cpu())
        e32 = rel_err(p32[n].grad.cpu(), p64[n].grad.cpu())
        report[n] = (round(e, 6), round(e32, 6))
    print("routed grad rel err (engine, torch fp32):", report)
    for n, (e, _) in report.items():
        assert e < ROUTED_GRAD_TOL, (n, e)


def test_dgcnn_eval_matches_oracle(golden, cuda):
    g = golden("dgcnn_small.npz")
    m = _dgcnn_from_golden(g, cuda)
    with torch.no_grad():
        for n, b in m.named_buffers():  # non-trivial running stats
            if n.endswith("running_mean"):
                b.copy_(torch.linspace(-0.2, 0.2, b.numel()))
            if n.endswith("running_var"):
                b.copy_(torch.linspace(0.5, 2.0, b.numel()))
    m.eval()
    x = torch.from_numpy(g["x"]).to(cuda)
    with torch.no_grad():
        y = m(x)
    params = {n: t.detach().cpu().clone() for n, t in m.state_dict().items()}
    ref, _ = R.dgcnn(torch.from_numpy(g["x"]), 10, params, training=False)
    assert rel_err(y.cpu(), ref) < TOL


def test_dgcnn_knn_bit_exact_per_layer(golden, cuda):
    """Each feature-space kNN inside the fused chain equals the oracle's kNN of
    the same (GPU-produced) features."""
    from dgx.edgeconv import edgeconv_stack
    g = golden("dgcnn_small.npz")
    m = _dgcnn_from_golden(g, cuda)
    x = torch.from_numpy(g["x"]).to(cuda)
    with torch.no_grad():
        feats = edgeconv_stack(x, 10, m.edge_blocks(), True).cpu()
    B, N = x.shape[0], x.shape[2]
    f = feats.view(B, N, -1)
    off = 0
    from models.dgcnn import knn
    for w in (64, 64, 128):
        xl = f[:, :, off:off + w].permute(0, 2, 1).contiguous()
        np.testing.assert_array_equal(knn(xl.to(cuda), 10).cpu().numpy(), oracle.knn(xl, 10))
        off += w


def test_dgcnn_state_dict_keys(golden):
    import json
    import os
    from conftest import GOLDEN
    from models.dgcnn import DGCNN
    from models.layers import PositionEmbedding
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        keys = json.load(f)["state_dict_keys"]
    assert list(DGCNN(types.SimpleNamespace(emb_dim=1024, k=20)).state_dict().keys()) == keys["DGCNN"]
    assert list(PositionEmbedding(types.SimpleNamespace(k=20)).state_dict().keys()) == keys["PositionEmbedding"]


def test_position_embedding_golden(golden, cuda):
    import hashlib
    from models.layers import PositionEmbedding
    g = golden("posemb_small.npz")
    torch.manual_seed(5)
    m = PositionEmbedding(types.SimpleNamespace(k=10))
    with torch.no_grad():
        m.transform.weight.normal_(0, 0.05)
    sha = hashlib.sha256(b"".join(v.detach().numpy().tobytes() for v in m.state_dict().values())).hexdigest()
    assert sha == str(g["init_sha256"])
    m = m.to(cuda).train()
    x = torch.from_numpy(g["x"]).to(cuda)
    y = m(x)
    assert rel_err(y.detach().cpu(), g["out"]) < TOL
    y.backward(torch.from_numpy(g["gout"]).to(cuda))
    # parameters whose true gradient is ~0 (bn3.bias: a BatchNorm1d follows the
    # max over points) are compared against the model-wide gradient scale
    gscale = max(np.abs(g[k]).max() for k in g.files if k.startswith("grad."))
    for n, p in m.named_parameters():
        key = "grad." + n
        if key in g.files:
            ref = g[key]
            err = np.abs(p.grad.cpu().numpy() - ref).max()
            assert err <= TOL * max(np.abs(ref).max(), 1e-3 * gscale) or frac_close(p.grad.cpu(), ref) >= 0.99, n
        elif "gradproj." + n in g.files:
            from dgx import synth
            r = synth.uniform(53, tuple(p.shape)) - 0.5
            proj = g["gradproj." + n]
            got = p.grad.cpu().double().numpy()
            assert abs((got * r).sum() - proj[0]) <= TOL * abs(proj[1]) * np.sqrt(r.size) * 0.3 + 1e-9, n
            assert abs(np.linalg.norm(got) - proj[1]) <= TOL * proj[1], n


def test_dgcnn_full_size_train_step(cuda):
    """cfg2 shape: finite outputs/grads, BN running stats move, and the chain's
    layer-1 kNN equals the oracle's at full size."""
    import oracle as O
    from models.dgcnn import DGCNN
    from dgx import synth
    torch.manual_seed(0)
    m = DGCNN(types.SimpleNamespace(emb_dim=1024, k=20)).to(cuda).train()
    pts = synth.cube_clouds(32, 1024, 0)
    with Capture() as cap:
        y = m(torch.from_numpy(pts).to(cuda).permute(0, 2, 1))
    assert tuple(y.shape) == (32, 1024, 1024)
    y.sum().backward()
    assert torch.isfinite(y).all()
    for p in m.parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all()
    assert float(m.conv1[1].running_var.mean()) != 1.0
    idx1 = cap[("fwd", 0)][0].cpu().numpy()
    want = O.knn(torch.from_numpy(pts).permute(0, 2, 1), 20)
    np.testing.assert_array_equal(idx1, want)


@pytest.mark.parametrize("B,N,k,emb,in_dims", [(32, 1024, 20, 1024, 3),    # cfg2: the bench headline
                                               (2, 2048, 40, 1024, 3),     # cfg3 geometry (bench --config cfg3)
                                               (2, 4096, 20, 1024, 9)])    # cfg5 model, S3DIS blocks
def test_dgcnn_bf16_headline_cfg2_routed(cuda, B, N, k, emb, in_dims):
    """The headline configuration (BASELINE configs[1]: DGCNN(emb 1024), B 32,
    N 1024, k 20, bf16 GEMMs) at full size, the cfg3 geometry (N 2048, k 40;
    two clouds of the 32), and the cfg5 model bench.py
    --config cfg5 times (DGCNN(in_dims=9) on S3DIS blocks, N 4096, k 20; two
    clouds of the per-GPU 24): train-mode output and every parameter gradient
    within SURVEY §8(c)'s bf16 bar (2e-2) of the fp64 oracle routed by the
    engine's own decisions."""
    from dgx import precision, synth
    from models.dgcnn import DGCNN
    torch.manual_seed(0)
    m = DGCNN(types.SimpleNamespace(emb_dim=emb, k=k, in_dims=in_dims))
    init = {n: t.detach().clone() for n, t in m.state_dict().items()}
    m = m.to(cuda).train()
    pts = _clouds(B, N, in_dims, 0 if in_dims == 3 else 2)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
    gout = torch.from_numpy(synth.uniform(1234, (B, emb, N)) - 0.5).float()
    precision.set("bf16")
    try:
        with Capture() as cap:
            y = m(x)
        y.backward(gout.to(cuda))
    finally:
        precision.set("fp32")
    print("decision check (gap, flip):", validate_dgcnn_decisions(cap, x, k, init, bf16=True))
    dec = [(i.long(), a, z) for (i, a, z) in (cap[("fwd", l)] for l in range(4))]
    params = {n: (t.to(cuda).double() if t.is_floating_point() else t.to(cuda)) for n, t in init.items()}
    for n, t in params.items():
        if t.is_floating_point() and "running" not in n:
            t.requires_grad_(True)
    ref = R.dgcnn_routed(torch.from_numpy(pts).to(cuda).double().permute(0, 2, 1), params, dec, y.detach() > 0)
    ref.backward(gout.to(cuda).double())
    errs = {"out": rel_err(y.detach().cpu(), ref.detach().cpu())}
    for n, p in m.named_parameters():
        errs[n] = rel_err(p.grad.cpu(), params[n].grad.cpu())
    print("bf16 cfg2 rel err:", {n: round(e, 5) for n, e in errs.items()})
    for n, e in errs.items():
        assert e < 2e-2, (n, e)


def test_dgcnn_bf16_mode_routed(cuda):
    """bf16 GEMM operands (BASELINE cfg2 precision), small emb: output and
    gradients within SURVEY §8(c)'s bf16 bar (2e-2) of the fp64 routed oracle."""
    from dgx import precision, synth
    from models.dgcnn import DGCNN
    torch.manual_seed(7)
    emb, N, k, B = 256, 512, 20, 2
    m = DGCNN(types.SimpleNamespace(emb_dim=emb, k=k))
    init = {n: t.detach().clone() for n, t in m.state_dict().items()}
    m = m.to(cuda).train()
    pts = synth.cube_clouds(B, N, 77)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
    precision.set("bf16")
    try:
        with Capture() as cap:
            y = m(x)
        gout = torch.from_numpy(synth.uniform(78, tuple(y.shape)) - 0.5)
        y.backward(gout.to(cuda))
    finally:
        precision.set("fp32")
    validate_dgcnn_decisions(cap, x, k, init, bf16=True)
    decisions = [tuple(t.cpu() for t in cap[("fwd", l)]) for l in range(4)]
    decisions = [(i.long(), a, z) for (i, a, z) in decisions]
    params = {n: (t.double() if t.is_floating_point() else t) for n, t in init.items()}
    for n, t in params.items():
        if t.is_floating_point() and "running" not in n:
            t.requires_grad_(True)
    ref = R.dgcnn_routed(torch.from_numpy(pts).double().permute(0, 2, 1), params, decisions, y.detach().cpu() > 0)
    ref.backward(gout.double())
    assert rel_err(y.detach().cpu(), ref.detach()) < 2e-2
    for n, p in m.named_parameters():
        assert rel_err(p.grad.cpu(), params[n].grad) < 2e-2, n


def test_dgcnn_large_n_generic_knn(cuda, monkeypatch):
    """A cloud larger than the fused kNN kernel's N (12288): every block's kNN
    takes the generic kernel, no block writes a fused kNN image for the next
    (ADVICE r04), in both dispatch paths (the one-op C++ layer and the
    autograd Functions), bit-equal to each other, with block 1's neighbours
    equal to the oracle's and finite gradients."""
    import oracle as O
    from dgx import host, ops, synth
    from models.dgcnn import DGCNN
    B, N, k = 1, 16384, 20
    assert not ops.fast_shape(3, k, N)
    torch.manual_seed(11)
    base = DGCNN(types.SimpleNamespace(emb_dim=64, k=k))
    pts = synth.cube_clouds(B, N, 17)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
    outs = []
    for enabled in (True, False):
        monkeypatch.setattr(host, "ENABLED", enabled)
        m = copy.deepcopy(base).to(cuda).train()
        y = m(x)
        y.square().mean().backward()
        outs.append((y.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    assert torch.equal(outs[0][0], outs[1][0])
    for n in outs[0][1]:
        assert torch.equal(outs[0][1][n], outs[1][1][n]), n
        assert torch.isfinite(outs[0][1][n]).all(), n
    got = ops.knn(x, k).cpu().numpy()
    np.testing.assert_array_equal(got, O.knn(torch.from_numpy(pts).permute(0, 2, 1), k))
