"""Mixed precision (autocast) and BatchNorm-mode contracts of the engine.

* main_partseg_dist.py:221,253 runs Net under torch.cuda.amp.autocast. The
  engine's GEMMs follow autocast without computing narrower than it (SURVEY
  §8(b), dgx.precision.effective): bf16 autocast takes the bf16 MFMA path and
  must equal precision "bf16" without autocast bit for bit (bf16 bar against
  the fp64 routed oracle); fp16 autocast takes the split-bf16 fp32 GEMMs (16
  significant bits per operand, finer than fp16's 11) and must equal precision
  "fp32_split" bit for bit (split bar). kNN, BN and the elementwise stages stay
  fp32, and every kernel must receive the dtype its C ABI declares
  (dgx._native.ptr asserts it).
* nn.BatchNorm decides batch vs running statistics per module; the engine must
  follow each BN's own flag (model.train() with frozen BN layers), and support
  backward through running-statistics BN, as the reference's autograd does.

The fp64 routed oracle (oracle/reference.py) runs on the GPU in float64 here:
the same ATen op sequence as on the CPU, only faster at cfg4 geometry.
"""
import threading
import types

import numpy as np
import pytest
import torch

from conftest import rel_err, validate_dgcnn_decisions
from oracle import reference as R

pytestmark = pytest.mark.gpu
TOL = 1e-3
TOL_BF16 = 2e-2   # bf16 GEMM operands (autocast / precision "bf16"): the headline bar
TOL_SPLIT = 5e-3  # split-bf16 GEMMs (fp16 autocast / precision "fp32_split"), ~2^-16 per product


class Capture:
    def __enter__(self):
        import dgx.edgeconv as E
        self.E = E
        E.set_debug_capture({})
        return E.debug_capture()

    def __exit__(self, *exc):
        self.E.set_debug_capture(None)


def _routed_oracle(init, pts, decisions, mask5, gout, dev, training=(True,) * 5):
    params = {n: (t.to(dev).double() if t.is_floating_point() else t.to(dev)) for n, t in init.items()}
    for n, t in params.items():
        if t.is_floating_point() and "running" not in n:
            t.requires_grad_(True)
    dec = [(i.to(dev).long(), a.to(dev), z.to(dev)) for (i, a, z) in decisions]
    x = torch.from_numpy(pts).to(dev).double().permute(0, 2, 1)
    ref = R.dgcnn_routed(x, params, dec, mask5.to(dev), training=training)
    ref.backward(gout.to(dev).double())
    return ref.detach(), params


def _decisions(cap):
    return [tuple(t for t in cap[("fwd", l)]) for l in range(4)]


@pytest.mark.parametrize("dtype", ["float16", "bfloat16"])
def test_dgcnn_autocast_cfg4_geometry(cuda, dtype):
    """DGCNN(emb 512, k 40) at N 2048 (BASELINE cfg4 / main_partseg_dist.py
    geometry, B reduced to 4) under torch.autocast: identical to the same model
    in the precision that autocast dtype maps to without autocast (fp16 ->
    "fp32_split", bf16 -> "bf16"; both dispatch paths), every routing decision
    the reference's own, and within that precision's bar of the fp64 routed
    oracle."""
    from dgx import precision as prec
    from dgx import synth
    from models.dgcnn import DGCNN
    dt = getattr(torch, dtype)
    mode, tol = ("fp32_split", TOL_SPLIT) if dt is torch.float16 else ("bf16", TOL_BF16)
    torch.manual_seed(4)
    B, N, k, emb = 4, 2048, 40, 512
    m = DGCNN(types.SimpleNamespace(emb_dim=emb, k=k))
    init = {n: t.detach().clone() for n, t in m.state_dict().items()}
    m = m.to(cuda).train()
    pts = synth.cube_clouds(B, N, 404)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
    gout = torch.from_numpy(synth.uniform(405, (B, emb, N)) - 0.5).float()
    with Capture() as cap:
        with torch.autocast("cuda", dtype=dt):
            y = m(x)
    assert y.dtype == torch.float32
    y.backward(gout.to(cuda))
    g_amp = {n: p.grad.clone() for n, p in m.named_parameters()}
    rs_amp = {n: b.clone() for n, b in m.named_buffers()}
    # the same step in the mapped precision without autocast (the one-op C++
    # path), and under autocast again through it: the same arithmetic
    for amp in (False, True):
        m.load_state_dict({n: t.to(cuda) for n, t in init.items()})
        m.zero_grad(set_to_none=True)
        if amp:
            with torch.autocast("cuda", dtype=dt):
                y2 = m(x)
        else:
            with prec.mode(mode):
                y2 = m(x)
        y2.backward(gout.to(cuda))
        assert torch.equal(y, y2)
        for n, p in m.named_parameters():
            assert torch.equal(p.grad, g_amp[n]), n
        for n, b in m.named_buffers():
            assert torch.equal(b, rs_amp[n]), n
    # every neighbour set (blocks 1-4) and every max slot / sign is the reference's own
    print("decision check (gap, flip):", validate_dgcnn_decisions(cap, x, k, init, bf16=mode == "bf16"))
    ref, params = _routed_oracle(init, pts, _decisions(cap), y.detach() > 0, gout, cuda)
    errs = {"y": rel_err(y.detach().cpu(), ref.cpu())}
    for n, p in m.named_parameters():
        errs[n] = rel_err(g_amp[n].cpu(), params[n].grad.cpu())
    print(dtype, mode, {n: f"{e:.1e}" for n, e in errs.items()})
    for n, e in errs.items():
        assert e < tol, (n, e)


def test_dgcnn_half_input(cuda):
    """An fp16 input (e.g. features produced under autocast) is up-cast: the
    result equals the engine's result on the same values in fp32."""
    from dgx import synth
    from models.dgcnn import DGCNN
    torch.manual_seed(1)
    m = DGCNN(types.SimpleNamespace(emb_dim=128, k=20)).to(cuda).eval()
    x = torch.from_numpy(synth.cube_clouds(2, 512, 9)).to(cuda).permute(0, 2, 1).half()
    with torch.no_grad():
        assert torch.equal(m(x), m(x.float()))


def test_position_embedding_autocast(cuda):
    """PositionEmbedding (k 40, N 2048) under autocast: the engine's edge stage
    follows the autocast dtype without computing narrower than it (bf16
    autocast: bit-equal to precision "bf16", within the bf16 bar of the fp32
    run; fp16 autocast: the exact fp32 kernels, bit-equal to the fp32 run); the
    stock layers after it (conv3, MLP, bmm) run in fp16 as in the reference. In
    eval mode (running statistics: a smooth function of the input) the module
    output stays within reduced-precision rounding of the fp32 run; in train
    mode backward completes, finite."""
    from dgx import precision as prec
    from dgx import synth
    from dgx.edgemlp import edge_mlp2
    from models.layers import PositionEmbedding
    torch.manual_seed(2)
    m = PositionEmbedding(types.SimpleNamespace(k=40))
    with torch.no_grad():
        m.transform.weight.normal_(0, 0.05)
    state = {n: t.clone() for n, t in m.state_dict().items()}
    m = m.to(cuda).train()
    x = torch.from_numpy(synth.cube_clouds(4, 2048, 11)).to(cuda).permute(0, 2, 1).contiguous().requires_grad_(True)

    def edge(dt=None, mode="fp32"):
        m.load_state_dict({n: t.to(cuda) for n, t in state.items()})
        with torch.autocast("cuda", dtype=dt or torch.float16, enabled=dt is not None), prec.mode(mode):
            return edge_mlp2(x, 40, m.conv1, m.conv2)
    e_h, e_b = edge(torch.float16), edge(torch.bfloat16)
    e16, e32 = edge(mode="bf16"), edge()
    assert e_h.dtype == torch.float32 and e_b.dtype == torch.float32
    assert torch.equal(e_h, e32) and torch.equal(e_b, e16)
    assert rel_err(e_b.detach().cpu(), e32.detach().cpu()) < TOL_BF16
    m.load_state_dict({n: t.to(cuda) for n, t in state.items()})
    with torch.autocast("cuda", dtype=torch.float16):
        y = m(x)
    y.float().sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)
    m.eval()
    with torch.no_grad():
        with torch.autocast("cuda", dtype=torch.float16):
            y16 = m(x)
        y32 = m(x)
    assert rel_err(y16.float().cpu(), y32.cpu()) < TOL_BF16


def test_net_autocast_grad_scaler(cuda):
    """Net (partseg) train step exactly as main_partseg_dist.py:239-265 drives
    it: autocast forward, GradScaler-scaled backward, scaler.step."""
    from dgx import synth
    from models.model_partseg import Net
    torch.manual_seed(3)
    args = types.SimpleNamespace(k=20, emb_dim=64, n_heads=4, n_blocks=1, ff_dims=128, dropout=0.0, nclasses=50)
    net = Net(args).to(cuda).train()
    opt = torch.optim.SGD(net.parameters(), lr=0.01)
    scaler = torch.amp.GradScaler("cuda")
    src = torch.from_numpy(synth.cube_clouds(2, 256, 12)).to(cuda).permute(0, 2, 1).contiguous()
    lbl = torch.nn.functional.one_hot(torch.tensor([3, 7]), 16).float().to(cuda)
    target = torch.randint(0, 50, (2, 256), device=cuda)
    with torch.autocast("cuda", dtype=torch.float16):
        out = net(src, lbl)
        loss = torch.nn.functional.cross_entropy(out.float(), target)
    scaler.scale(loss).backward()
    scaler.step(opt)
    scaler.update()
    assert torch.isfinite(loss)
    assert all(torch.isfinite(p.grad).all() for p in net.emb_nn.parameters())


def test_edgeconv_eval_mode_backward(cuda):
    """Backward through a running-statistics (eval) EdgeConv block, as the
    reference's autograd supports: outputs and all gradients within 1e-3 of the
    fp64 routed oracle with BN in eval mode; running statistics untouched."""
    from dgx.edgeconv import edgeconv_stack
    torch.manual_seed(8)
    B, C, Co, N, k = 2, 64, 128, 512, 20
    blk = torch.nn.Sequential(torch.nn.Conv2d(2 * C, Co, 1, bias=False), torch.nn.BatchNorm2d(Co),
                              torch.nn.LeakyReLU(0.2, inplace=True))
    with torch.no_grad():
        blk[1].weight.copy_(torch.randn(Co))
        blk[1].bias.copy_(0.1 * torch.randn(Co))
        blk[1].running_mean.copy_(0.3 * torch.randn(Co))
        blk[1].running_var.copy_(torch.rand(Co) + 0.5)
    state = {n: t.clone() for n, t in blk.state_dict().items()}
    blk = blk.to(cuda).eval()
    x = torch.randn(B, C, N)
    xg = x.to(cuda).requires_grad_(True)
    with Capture() as cap:
        out = edgeconv_stack(xg, k, [blk]).view(B, N, Co).permute(0, 2, 1)
    gout = torch.randn(B, Co, N)
    out.backward(gout.to(cuda))
    idx, arg, zpos = cap[("fwd", 0)]
    xc = x.double().requires_grad_(True)
    wc = state["0.weight"].double().requires_grad_(True)
    gc = state["1.weight"].double().requires_grad_(True)
    bc = state["1.bias"].double().requires_grad_(True)
    bn = {"weight": gc, "bias": bc, "running_mean": state["1.running_mean"].double(),
          "running_var": state["1.running_var"].double()}
    ref, _ = R.edgeconv_block_routed(xc, wc, bn, idx.cpu().long(), arg.cpu(), zpos.cpu(), training=False)
    ref.backward(gout.double())
    assert rel_err(out.detach().cpu(), ref.detach()) < TOL
    for got, want in ((xg.grad, xc.grad), (blk[0].weight.grad, wc.grad), (blk[1].weight.grad, gc.grad),
                      (blk[1].bias.grad, bc.grad)):
        assert rel_err(got.cpu(), want) < TOL
    assert torch.equal(blk[1].running_mean.cpu(), state["1.running_mean"])
    assert torch.equal(blk[1].running_var.cpu(), state["1.running_var"])
    assert int(blk[1].num_batches_tracked) == 0


def test_dgcnn_frozen_bn_layers(cuda):
    """model.train() with conv2's and conv5's BatchNorm frozen in eval(): those
    layers normalise with (and keep) their running statistics, the others use
    batch statistics — nn.BatchNorm's per-module rule — in output, gradients and
    buffers (1e-3 against the fp64 routed oracle)."""
    from dgx import synth
    from models.dgcnn import DGCNN
    torch.manual_seed(6)
    B, N, k, emb = 2, 1024, 20, 256
    m = DGCNN(types.SimpleNamespace(emb_dim=emb, k=k))
    with torch.no_grad():
        for name in ("conv2", "conv5"):
            bn = getattr(m, name)[1]
            bn.running_mean.copy_(0.2 * torch.randn(bn.num_features))
            bn.running_var.copy_(torch.rand(bn.num_features) + 0.5)
    init = {n: t.detach().clone() for n, t in m.state_dict().items()}
    m = m.to(cuda).train()
    m.conv2[1].eval()
    m.conv5[1].eval()
    pts = synth.cube_clouds(B, N, 66)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
    with Capture() as cap:
        y = m(x)
    gout = torch.from_numpy(synth.uniform(67, tuple(y.shape)) - 0.5).float()
    y.backward(gout.to(cuda))
    flags = (True, False, True, True, False)
    validate_dgcnn_decisions(cap, x, k, init, training=flags[:4])
    ref, params = _routed_oracle(init, pts, _decisions(cap), y.detach() > 0, gout, cuda, training=flags)
    assert rel_err(y.detach().cpu(), ref.cpu()) < TOL
    for n, p in m.named_parameters():
        assert rel_err(p.grad.cpu(), params[n].grad.cpu()) < TOL, n
    for n, b in m.state_dict().items():
        if "running" in n:
            assert rel_err(b.cpu(), params[n].cpu()) < 1e-5, n
    assert int(m.conv2[1].num_batches_tracked) == 0 and int(m.conv1[1].num_batches_tracked) == 1


def test_edge_mlp_eval_mode_backward(cuda):
    """PositionEmbedding's edge stage with both BatchNorms in eval mode and the
    output differentiated: gradients match the fp64 reference module (eval)."""
    from dgx import synth
    from dgx.edgemlp import edge_mlp2
    from oracle import knn as oknn
    B, N, k = 2, 300, 16
    g = torch.Generator().manual_seed(12)

    def block(ci, co):
        blk = torch.nn.Sequential(torch.nn.Conv2d(ci, co, 1, bias=False), torch.nn.BatchNorm2d(co),
                                  torch.nn.LeakyReLU(0.2))
        with torch.no_grad():
            blk[0].weight.copy_(torch.randn(co, ci, 1, 1, generator=g) / np.sqrt(ci))
            gam = 1.0 + 0.3 * torch.randn(co, generator=g)
            gam[::5] *= -1.0
            blk[1].weight.copy_(gam)
            blk[1].bias.copy_(0.2 * torch.randn(co, generator=g))
            blk[1].running_mean.copy_(0.2 * torch.randn(co, generator=g))
            blk[1].running_var.copy_(torch.rand(co, generator=g) + 0.5)
        return blk
    c1, c2 = block(6, 64), block(64, 128)
    r1 = torch.nn.Sequential(torch.nn.Conv2d(6, 64, 1, bias=False), torch.nn.BatchNorm2d(64), torch.nn.LeakyReLU(0.2))
    r2 = torch.nn.Sequential(torch.nn.Conv2d(64, 128, 1, bias=False), torch.nn.BatchNorm2d(128),
                             torch.nn.LeakyReLU(0.2))
    r1.load_state_dict(c1.state_dict())
    r2.load_state_dict(c2.state_dict())
    r1, r2 = r1.double().eval(), r2.double().eval()
    c1, c2 = c1.to(cuda).eval(), c2.to(cuda).eval()
    pts = synth.cube_clouds(B, N, 13)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1).requires_grad_(True)
    y = edge_mlp2(x, k, c1, c2)
    gout = torch.from_numpy(synth.uniform(14, (B, 128, N)) - 0.5).float()
    y.backward(gout.to(cuda))
    x64 = torch.from_numpy(pts).double().permute(0, 2, 1).requires_grad_(True)
    idx = torch.as_tensor(oknn(torch.from_numpy(pts).permute(0, 2, 1), k)).long()
    ref = r2(r1(R.graph_feature(x64, k, idx=idx))).max(dim=-1)[0]
    ref.backward(gout.double())
    assert rel_err(y.detach().cpu(), ref.detach()) < TOL
    pairs = [(x.grad, x64.grad)]
    for got, want in ((c1, r1), (c2, r2)):
        pairs += [(got[0].weight.grad, want[0].weight.grad), (got[1].weight.grad, want[1].weight.grad),
                  (got[1].bias.grad, want[1].bias.grad)]
    for got, want in pairs:
        assert rel_err(got.cpu(), want) < TOL
    assert int(c1[1].num_batches_tracked) == 0


def test_concurrent_threads(cuda):
    """nn.DataParallel runs replicas in Python threads (main_cls.py:62,
    torch/nn/parallel/parallel_apply.py): two threads driving DGCNN train steps
    through the engine at once, each on its own stream, give the results of the
    same steps run one after the other (no shared mutable engine state)."""
    from dgx import synth
    from models.dgcnn import DGCNN
    torch.manual_seed(10)
    base = DGCNN(types.SimpleNamespace(emb_dim=128, k=20))
    models = [DGCNN(types.SimpleNamespace(emb_dim=128, k=20)) for _ in range(2)]
    for mm in models:
        mm.load_state_dict(base.state_dict())
    xs = [torch.from_numpy(synth.cube_clouds(4, 1024, 20 + i)).to(cuda).permute(0, 2, 1) for i in range(2)]

    def run(mm, x, out, i):
        stream = torch.cuda.Stream(cuda)
        with torch.cuda.stream(stream):
            mm = mm.to(cuda).train()
            y = None
            for _ in range(3):
                mm.zero_grad(set_to_none=True)
                y = mm(x)
                y.square().mean().backward()
        stream.synchronize()
        out[i] = (y.detach().clone(), {n: p.grad.clone() for n, p in mm.named_parameters()})

    seq = {}
    for i in range(2):
        m2 = DGCNN(types.SimpleNamespace(emb_dim=128, k=20))
        m2.load_state_dict(base.state_dict())
        run(m2, xs[i], seq, i)
    par = {}
    threads = [threading.Thread(target=run, args=(models[i], xs[i], par, i)) for i in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    for i in range(2):
        assert torch.equal(par[i][0], seq[i][0])
        for n in seq[i][1]:
            assert torch.equal(par[i][1][n], seq[i][1][n]), n
