"""Fused edge-MLP backward (dgx_edge_mlp_fused_bwd_bf16; PositionEmbedding's
conv2 + LReLU/BN1 backward, reference models/layers.py:48-52 under autograd)
against the unfused bf16 path it replaces (dZ2 GEMM with the BN2 backward in
its epilogue, dH1 GEMM with the LReLU/BN1 backward in its epilogue, dW2 =
dZ2^T H1 GEMM over the h1 the forward stored).

Both paths round the same operands to bf16 at the same points (h1, dZ2, gE) and
differ only in fp32 summation order (dH1 over c2 in two halves, dW2 over edges
per block), so a handful of bf16 ulps in gE is the whole difference: every
gradient within TOL normwise. The fp64 parity of the bf16 mode itself is
tests/test_edgemlp_gpu.py::test_edge_mlp_bf16_mode (now running the fused
backward)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 5e-3  # normwise, fused vs unfused bf16 backward


def _convs(seed):
    torch.manual_seed(seed)
    c1 = torch.nn.Sequential(torch.nn.Conv2d(6, 64, 1, bias=False), torch.nn.BatchNorm2d(64),
                             torch.nn.LeakyReLU(0.2))
    c2 = torch.nn.Sequential(torch.nn.Conv2d(64, 128, 1, bias=False), torch.nn.BatchNorm2d(128),
                             torch.nn.LeakyReLU(0.2))
    with torch.no_grad():
        for bn in (c1[1], c2[1]):
            bn.weight.copy_(torch.randn(bn.weight.shape))  # negative gammas too
            bn.bias.copy_(0.1 * torch.randn(bn.bias.shape))
    return c1, c2


def _run(cuda, B, N, k, fused, seed=5):
    import dgx.edgemlp as EM
    from dgx import precision, synth
    conv1, conv2 = _convs(seed)
    conv1, conv2 = conv1.to(cuda).train(), conv2.to(cuda).train()
    x = torch.from_numpy(synth.cube_clouds(B, N, seed)).to(cuda).permute(0, 2, 1).requires_grad_(True)
    gout = torch.from_numpy(synth.uniform(seed + 1, (B, 128, N)) - 0.5).float().to(cuda)
    precision.set("bf16")
    old = EM.FUSED_BWD
    EM.FUSED_BWD = fused
    try:
        y = EM.edge_mlp2(x, k, conv1, conv2, True)
        y.backward(gout)
    finally:
        EM.FUSED_BWD = old
        precision.set("fp32")
    grads = {"x": x.grad, "w1": conv1[0].weight.grad, "g1": conv1[1].weight.grad, "b1": conv1[1].bias.grad,
             "w2": conv2[0].weight.grad, "g2": conv2[1].weight.grad, "b2": conv2[1].bias.grad}
    return y.detach(), {n: g.detach().double().cpu() for n, g in grads.items()}


@pytest.mark.parametrize("B,N,k", [(2, 1024, 40), (2, 512, 20), (3, 300, 33), (1, 130, 9), (4, 2048, 40)])
def test_fused_backward_matches_unfused(cuda, B, N, k):
    y1, g1 = _run(cuda, B, N, k, True)
    y0, g0 = _run(cuda, B, N, k, False)
    assert torch.equal(y1, y0)  # same forward kernel either way
    errs = {n: float((g1[n] - g0[n]).norm() / g0[n].norm()) for n in g0}
    print("fused vs unfused bwd rel err:", {n: f"{e:.1e}" for n, e in errs.items()})
    assert all(e < TOL for e in errs.values()), errs


def test_fused_backward_skips_h1_store(cuda):
    """With the fused backward the forward keeps no h1 (E x 64 bf16) for autograd."""
    import dgx.edgemlp as EM
    from dgx import precision, synth
    conv1, conv2 = _convs(3)
    conv1, conv2 = conv1.to(cuda).train(), conv2.to(cuda).train()
    x = torch.from_numpy(synth.cube_clouds(2, 256, 3)).to(cuda).permute(0, 2, 1).requires_grad_(True)
    precision.set("bf16")
    try:
        y = EM.edge_mlp2(x, 20, conv1, conv2, True)
    finally:
        precision.set("fp32")
    saved = y.grad_fn.saved_tensors  # the engine Function's own node (it returns its output)
    assert len(saved) == 10
    assert all(t is None or t.shape[0] != 2 * 256 * 20 for t in saved)
