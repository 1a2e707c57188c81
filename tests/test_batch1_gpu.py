"""B = 1 with a channel-major (1, C, N) input, the layout the reference's
modules receive (models/layers.py:45, models/dgcnn.py:76): the point-major
view x.permute(0, 2, 1).reshape(N, C) is then a column-major VIEW, not a copy,
and must still reach the GEMMs as row-major rows. Output and gradients equal
those of the same values stored point-major."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _inputs(cuda, N, seed):
    g = torch.Generator().manual_seed(seed)
    x_cm = (torch.rand(1, 3, N, generator=g) * 2 - 1).to(cuda)                # channel-major storage
    x_pm = x_cm.permute(0, 2, 1).contiguous().permute(0, 2, 1)              # same values, point-major
    return x_cm.requires_grad_(True), x_pm.requires_grad_(True)


def _seq(cin, cout, seed, conv2d=True):
    torch.manual_seed(seed)
    conv = torch.nn.Conv2d(cin, cout, 1, bias=False) if conv2d else torch.nn.Conv1d(cin, cout, 1, bias=False)
    return torch.nn.Sequential(conv, torch.nn.BatchNorm2d(cout), torch.nn.LeakyReLU(0.2))


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_edge_mlp_batch1_channel_major(cuda, mode):
    import dgx.edgemlp as EM
    from dgx import precision
    res = []
    for which in range(2):
        c1, c2 = _seq(6, 64, 1).to(cuda).train(), _seq(64, 128, 2).to(cuda).train()
        x = _inputs(cuda, 77, 3)[which]
        precision.set(mode)
        try:
            y = EM.edge_mlp2(x, 20, c1, c2, True)
            y.backward(torch.ones_like(y))
        finally:
            precision.set("fp32")
        res.append((y.detach(), x.grad, c1[0].weight.grad, c2[0].weight.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_edgeconv_batch1_channel_major(cuda):
    from dgx.edgeconv import edgeconv_stack_pair
    res = []
    for which in range(2):
        convs = [_seq(6, 64, 4).to(cuda).train()]
        x = _inputs(cuda, 90, 5)[which]
        y, _ = edgeconv_stack_pair(x, 16, convs)
        y.backward(torch.ones_like(y))
        res.append((y.detach(), x.grad, convs[0][0].weight.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)
