"""f2: the engine attention (csrc/attention.hip via dgx.attention) against an
fp64 restatement of scaled_dot_product_attention (the op nn.MultiheadAttention
runs inside the reference's Net, models/model_partseg.py:167-171, 187-191) on
the same 16-bit-rounded operands, with the kernels' own dropout mask.

Tolerances are normwise (max |err| / max |ref|): the kernels round P (and dS in
the backward) to the 16-bit operand type before their second MFMA and keep
every sum in fp32, so the error is a few units of that type's rounding.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# fp32: the split-plane mode (x = bf16 hi + bf16 lo, three MFMAs per product)
TOL_FWD = {torch.float16: 2e-3, torch.bfloat16: 1.2e-2, torch.float32: 1e-4}
TOL_BWD = {torch.float16: 5e-3, torch.bfloat16: 3e-2, torch.float32: 2e-4}


def _nerr(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-30))


def _ref(q, k, v, heads, scale, mask=None, p=0.0):
    """fp64 attention on (B, N, E) operands; mask: (B*H*Nq, Nk) keep mask."""
    B, Nq, E = q.shape
    Nk = k.shape[1]
    D = E // heads
    qh = q.double().view(B, Nq, heads, D).transpose(1, 2)
    kh = k.double().view(B, Nk, heads, D).transpose(1, 2)
    vh = v.double().view(B, Nk, heads, D).transpose(1, 2)
    a = torch.softmax(qh @ kh.transpose(-1, -2) * scale, dim=-1)
    if mask is not None:
        a = a * mask.view(B, heads, Nq, Nk).double() / (1.0 - p)
    return (a @ vh).transpose(1, 2).reshape(B, Nq, E)


def _inputs(B, Nq, Nk, E, dt, dev, seed, strided=False):
    g = torch.Generator().manual_seed(seed)
    if strided:  # views of one (B, N, 3E) projection, as nn.MultiheadAttention makes them
        qkv = torch.randn((B, Nq, 3 * E), generator=g).to(dt).to(dev)
        return qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
    q = torch.randn((B, Nq, E), generator=g).to(dt).to(dev)
    k = torch.randn((B, Nk, E), generator=g).to(dt).to(dev)
    v = torch.randn((B, Nk, E), generator=g).to(dt).to(dev)
    return q, k, v


CASES = [  # B, heads, Nq, Nk, D
    (2, 4, 256, 256, 128),
    (1, 2, 77, 300, 128),
    (2, 3, 130, 64, 64),
    (1, 1, 1, 33, 64),
    (2, 4, 200, 200, 16),   # Net's test config head size (padded to 64)
]


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,H,Nq,Nk,D", CASES)
def test_attention_forward_backward(cuda, dt, B, H, Nq, Nk, D):
    from dgx.attention import attention
    E = H * D
    q, k, v = _inputs(B, Nq, Nk, E, dt, cuda, B * 7 + Nq + D)
    q.requires_grad_(True)
    k.requires_grad_(True)
    v.requires_grad_(True)
    o = attention(q, k, v, H)
    assert o.dtype == dt and o.shape == (B, Nq, E)
    assert q.dtype != torch.float32 or __import__("dgx.precision").precision.get() == "fp32"
    scale = 1.0 / math.sqrt(D)
    qr, kr, vr = (t.detach().double().requires_grad_(True) for t in (q, k, v))
    ref = _ref(qr, kr, vr, H, scale)
    assert _nerr(o, ref) < TOL_FWD[dt], _nerr(o, ref)
    go = torch.randn(o.shape, generator=torch.Generator().manual_seed(3)).to(dt).to(cuda)
    o.backward(go)
    ref.backward(go.double())
    for name, got, want in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        assert _nerr(got, want) < TOL_BWD[dt], (name, _nerr(got, want))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_attention_strided_projection_views(cuda, dt):
    """q/k/v as column slices of one (B, N, 3E) tensor run without a copy and
    give the same result as contiguous operands."""
    from dgx.attention import attention
    q, k, v = _inputs(2, 192, 192, 256, dt, cuda, 11, strided=True)
    o1 = attention(q, k, v, 2)
    o2 = attention(q.contiguous(), k.contiguous(), v.contiguous(), 2)
    torch.testing.assert_close(o1, o2, rtol=0, atol=0)


@pytest.mark.parametrize("p,dt", [(0.5, torch.float16), (0.1, torch.float16), (0.5, torch.float32)])
def test_attention_dropout_matches_masked_reference(cuda, monkeypatch, p, dt):
    """Forward and backward with dropout equal the fp64 reference that applies
    the kernels' own keep mask (dgx_attn_dropout_mask) to the softmax weights."""
    import dgx.attention as A
    B, H, N, D = 2, 4, 160, 64
    E = H * D
    seed = 0x1234_5678_9ABC
    monkeypatch.setattr(A, "new_seed", lambda dev: torch.tensor([seed], dtype=torch.int64, device=dev))
    q, k, v = _inputs(B, N, N, E, dt, cuda, 21)
    for t in (q, k, v):
        t.requires_grad_(True)
    o = A.attention(q, k, v, H, dropout_p=p)
    mask = A.dropout_mask(B * H * N, N, p, seed, cuda)
    qr, kr, vr = (t.detach().double().requires_grad_(True) for t in (q, k, v))
    ref = _ref(qr, kr, vr, H, 1.0 / math.sqrt(D), mask=mask, p=p)
    assert _nerr(o, ref) < TOL_FWD[dt]
    go = torch.randn(o.shape, generator=torch.Generator().manual_seed(5)).to(dt).to(cuda)
    o.backward(go)
    ref.backward(go.double())
    for got, want in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        assert _nerr(got, want) < TOL_BWD[dt]


def test_dropout_mask_statistics(cuda):
    from dgx.attention import dropout_mask
    for p in (0.5, 0.1, 0.9):
        m = dropout_mask(512, 2048, p, 99, cuda).double()
        assert abs(m.mean().item() - (1 - p)) < 2e-3, (p, m.mean().item())
        # rows and columns are not correlated: per-row keep rates spread like a binomial
        rows = m.mean(1)
        assert rows.std().item() < 3 * math.sqrt(p * (1 - p) / 2048)
    a = dropout_mask(64, 512, 0.5, 1, cuda)
    b = dropout_mask(64, 512, 0.5, 2, cuda)
    assert (a != b).double().mean().item() > 0.4
    assert dropout_mask(8, 64, 0.0, 1, cuda).all()


def test_attention_deterministic(cuda):
    from dgx.attention import attention
    q, k, v = _inputs(2, 256, 256, 256, torch.float16, cuda, 8)
    outs = []
    for _ in range(2):
        qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v))
        o = attention(qq, kk, vv, 2)
        o.sum().backward()
        outs.append((o, qq.grad, kk.grad, vv.grad))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["self", "cross", "separate"])
def test_engine_mha_matches_torch_mha(cuda, mode):
    """EngineMultiheadAttention (eval: no dropout) vs stock nn.MultiheadAttention
    with the same weights, under fp16 autocast as main_partseg_dist.py runs it."""
    from dgx.attention import EngineMultiheadAttention, use_engine_attention
    torch.manual_seed(0)
    E, H, B, N, M = 256, 2, 2, 128, 96
    ref = torch.nn.MultiheadAttention(E, H, dropout=0.5, batch_first=True).to(cuda).eval()
    eng = torch.nn.MultiheadAttention(E, H, dropout=0.5, batch_first=True).to(cuda).eval()
    eng.load_state_dict(ref.state_dict())
    use_engine_attention(eng)
    assert isinstance(eng, EngineMultiheadAttention)
    assert list(eng.state_dict()) == list(ref.state_dict())
    x = torch.randn(B, N, E, device=cuda)
    mem = torch.randn(B, M, E, device=cuda)
    args = {"self": (x, x, x), "cross": (x, mem, mem), "separate": (x, mem, mem.clone())}[mode]
    with torch.autocast("cuda", dtype=torch.float16):
        want, _ = ref(*args, need_weights=False)
        got, _ = eng(*args, need_weights=False)
    assert _nerr(got, want) < 5e-3
    with pytest.raises(NotImplementedError):
        eng(x, x, x)  # need_weights=True (the nn.MultiheadAttention default) is not served


def test_engine_mha_train_step(cuda):
    """Training mode (dropout 0.5) runs fwd + bwd through the engine with finite
    gradients on every parameter; p = 0 in training equals eval."""
    from dgx.attention import use_engine_attention
    torch.manual_seed(1)
    m = use_engine_attention(torch.nn.MultiheadAttention(128, 2, dropout=0.5, batch_first=True).to(cuda)).train()
    x = torch.randn(2, 64, 128, device=cuda, requires_grad=True)
    y, _ = m(x, x, x, need_weights=False)
    y.square().mean().backward()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())
    m.dropout = 0.0
    y_tr, _ = m(x, x, x, need_weights=False)
    y_ev, _ = m.eval()(x, x, x, need_weights=False)
    assert torch.equal(y_tr, y_ev)


def test_net_attention_on_engine(cuda):
    """Net's transformer and final attention run on the engine (row f2): every
    nn.MultiheadAttention inside Net is the engine class, an eval forward
    matches the same weights on stock PyTorch attention (fp32 parity mode),
    and a dropout-0.5 training step (the reference default) has finite grads."""
    import types
    from dgx import synth
    from dgx.attention import EngineMultiheadAttention
    from models.model_partseg import Net
    torch.manual_seed(4)
    args = types.SimpleNamespace(k=20, emb_dim=128, n_heads=2, n_blocks=1, ff_dims=128, dropout=0.5, nclasses=50)
    net = Net(args).to(cuda)
    mhas = [m for m in net.modules() if isinstance(m, torch.nn.MultiheadAttention)]
    assert len(mhas) == 4 and all(type(m) is EngineMultiheadAttention for m in mhas)
    src = torch.from_numpy(synth.cube_clouds(2, 512, 3)).to(cuda).permute(0, 2, 1).contiguous()
    lbl = torch.nn.functional.one_hot(torch.tensor([1, 9]), 16).float().to(cuda)
    net.eval()
    with torch.no_grad():
        got = net(src, lbl)
        for m in mhas:
            m.__class__ = torch.nn.MultiheadAttention
        want = net(src, lbl)
        for m in mhas:
            m.__class__ = EngineMultiheadAttention
    assert _nerr(got, want) < 1e-4, _nerr(got, want)
    net.train()
    out = net(src, lbl)
    out.square().mean().backward()
    for n, p in net.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), n


def test_dropout_seed_is_device_drawn_and_graph_safe(cuda):
    """The dropout seed comes from the device generator (dgx.attention.new_seed):
    the host RNG stream that shuffles / augmentations draw from is untouched, and
    a captured graph draws a new mask on every replay instead of baking one in."""
    from dgx.attention import attention
    B, H, N, D = 1, 2, 128, 64
    q, k, v = _inputs(B, N, N, H * D, torch.float16, cuda, 31)
    torch.manual_seed(0)
    host = torch.random.get_rng_state()
    o1 = attention(q, k, v, H, dropout_p=0.5)
    o2 = attention(q, k, v, H, dropout_p=0.5)
    assert torch.equal(torch.random.get_rng_state(), host)
    assert not torch.equal(o1, o2)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        attention(q, k, v, H, dropout_p=0.5)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = attention(q, k, v, H, dropout_p=0.5)
    g.replay()
    a = out.clone()
    g.replay()
    torch.cuda.synchronize()
    assert not torch.equal(a, out)


@pytest.mark.parametrize("batch_first", [True, False])
def test_mha_projection_form_follows_operand_identity(cuda, monkeypatch, batch_first):
    """Self-attention is one (B, N, 3E) in-projection and cross-attention over one
    memory one (B, M, 2E) projection, whatever batch_first is (the identity of
    the operands is taken before the sequence-first transpose)."""
    import dgx.attention as A
    m = A.EngineMultiheadAttention(128, 2, batch_first=batch_first).to(cuda).eval()
    calls = []
    lin = A.F.linear
    monkeypatch.setattr(A.F, "linear", lambda x, w, b=None: calls.append(tuple(w.shape)) or lin(x, w, b))
    x = torch.randn(2, 64, 128, device=cuda)
    mem = torch.randn(2, 96, 128, device=cuda)
    if not batch_first:
        x, mem = x.transpose(0, 1), mem.transpose(0, 1)
    with torch.no_grad():
        m(x, x, x, need_weights=False)
        assert calls[0] == (384, 128) and len(calls) == 2, calls
        calls.clear()
        m(x, mem, mem, need_weights=False)
        assert calls[:2] == [(128, 128), (256, 128)] and len(calls) == 3, calls
