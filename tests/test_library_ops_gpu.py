"""SURVEY §8(b) torch op layer: the engine as torch.ops.dgx custom ops (dgx.library).

* every op's result equals the engine's autograd-Function path bit for bit
  (the op's device kernel runs the same code);
* torch.compile(DGCNN, fullgraph=True) traces the train step with no graph
  break (the ops' fake kernels describe every output) and its forward,
  backward and BatchNorm buffer updates equal the eager engine's bit for bit;
* torch.export captures the eval forward.
The compiled runs use AOTAutograd's eager backend: the point is the graph
capture of the engine's ops, not a code generator for the glue around them.
"""
import copy
import types

import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _model(emb=128, k=20, seed=0):
    from models.dgcnn import DGCNN
    torch.manual_seed(seed)
    return DGCNN(types.SimpleNamespace(emb_dim=emb, k=k))


def _cloud(cuda, B=4, N=512, seed=5):
    from dgx import synth
    return torch.from_numpy(synth.cube_clouds(B, N, seed)).to(cuda).permute(0, 2, 1)


def _step(m, x, gout, call=None):
    """One train step; ``call``: the callable to run (e.g. the compiled module), m its parameters' owner."""
    m.zero_grad(set_to_none=True)
    y = (call if call is not None else m)(x)
    y.backward(gout)
    return (y.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()},
            {n: b.clone() for n, b in m.named_buffers()})


def _assert_same(a, b):
    assert torch.equal(a[0], b[0])
    for n in a[1]:
        assert torch.equal(a[1][n], b[1][n]), n
    for n in a[2]:
        assert torch.equal(a[2][n], b[2][n]), n


def test_knn_and_graph_feature_ops(cuda):
    import dgx.library  # noqa: F401  (registers torch.ops.dgx)
    from dgx import ops
    x = _cloud(cuda, 2, 300)
    idx = torch.ops.dgx.knn(x, 16)
    assert idx.dtype == torch.int64 and torch.equal(idx, ops.knn(x, 16))
    with torch.autocast("cuda", dtype=torch.float16):   # autocast rule: distances stay fp32
        assert torch.equal(torch.ops.dgx.knn(x, 16), idx)
    for mode in (0, 1, 2):
        xa = x.detach().clone().requires_grad_(True)
        xb = x.detach().clone().requires_grad_(True)
        out, _ = torch.ops.dgx.graph_feature(xa, 16, mode)
        ref = ops.graph_feature(xb, 16, knn_only=mode == 2, disp_only=mode == 1)
        assert torch.equal(out, ref)
        g = torch.randn_like(out)
        out.backward(g)
        ref.backward(g)
        # the edge-tensor backward scatter-adds with atomics: equal up to summation order
        assert rel_err(xa.grad.cpu(), xb.grad.cpu()) < 1e-6


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_dgcnn_op_path_equals_function_path(cuda, monkeypatch, precision):
    """DGCNN through torch.ops.dgx == through the autograd Functions: train
    step (output, every gradient, every BN buffer) and eval forward."""
    from dgx import library, precision as prec
    base = _model()
    x = _cloud(cuda)
    gout = torch.randn((4, 128, 512), device=cuda)
    prec.set(precision)
    try:
        ma, mb = copy.deepcopy(base).to(cuda).train(), copy.deepcopy(base).to(cuda).train()
        a = _step(ma, x, gout)
        monkeypatch.setattr(library, "ENABLED", False)
        b = _step(mb, x, gout)
        _assert_same(a, b)
        ma.eval()
        mb.eval()
        with torch.no_grad():
            eb = mb(x)
        monkeypatch.setattr(library, "ENABLED", True)
        with torch.no_grad():
            ea = ma(x)
        assert torch.equal(ea, eb)
    finally:
        prec.set("fp32")


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_torch_compile_dgcnn_fullgraph(cuda, precision):
    """torch.compile(DGCNN, fullgraph=True): no graph break at the engine, and
    two compiled train steps equal two eager ones bit for bit (outputs,
    gradients, running statistics, batch counters)."""
    from dgx import precision as prec
    base = _model(seed=3)
    x = _cloud(cuda, seed=9)
    gout = torch.randn((4, 128, 512), device=cuda)
    prec.set(precision)
    try:
        me = copy.deepcopy(base).to(cuda).train()
        mc = copy.deepcopy(base).to(cuda).train()
        compiled = torch.compile(mc, backend="aot_eager", fullgraph=True)
        for _ in range(2):
            e = _step(me, x, gout)
            c = _step(mc, x, gout, call=compiled)
            _assert_same(e, c)
        assert int(mc.conv1[1].num_batches_tracked) == 2
    finally:
        prec.set("fp32")
        torch._dynamo.reset()


def test_torch_export_dgcnn_eval(cuda):
    """torch.export of the eval forward: one graph over the dgx ops, equal to eager."""
    import dgx.library  # noqa: F401
    m = _model(seed=4).to(cuda).eval()
    x = _cloud(cuda, seed=2)
    ep = torch.export.export(m, (x.contiguous(),))
    targets = {str(n.target) for n in ep.graph.nodes if n.op == "call_function"}
    assert any("dgx.edgeconv_chain" in t for t in targets) and any("dgx.pointconv" in t for t in targets), targets
    with torch.no_grad():
        assert rel_err(ep.module()(x.contiguous()).cpu(), m(x.contiguous()).cpu()) == 0.0


def test_bn_cumulative_average_op_path(cuda, monkeypatch):
    """BatchNorm with momentum=None (nn.BatchNorm's cumulative moving average):
    the op layer's finalize reads num_batches_tracked on the device (no host
    read, so the step stays capturable) and three train steps leave the same
    running statistics and counters as the autograd-Function path, which
    updates the module buffers in place like nn.BatchNorm."""
    from dgx import library
    base = _model(seed=6)
    for m in base.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = None
    x = _cloud(cuda, seed=11)
    gout = torch.randn((4, 128, 512), device=cuda)
    ma, mb = copy.deepcopy(base).to(cuda).train(), copy.deepcopy(base).to(cuda).train()
    for _ in range(3):
        monkeypatch.setattr(library, "ENABLED", True)
        a = _step(ma, x, gout)
        monkeypatch.setattr(library, "ENABLED", False)
        b = _step(mb, x, gout)
        _assert_same(a, b)
    assert int(ma.conv1[1].num_batches_tracked) == 3
