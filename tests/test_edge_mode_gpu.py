"""The paper's edge feature (x_j - x_i, x_i) (reference test.ipynb:131; the
shipped models/dgcnn.py:42 uses (x_j, x_i)): get_graph_feature
mode="diff" and DGCNN edge_mode="diff" (the same engine kernels on the
re-parameterised weight [W1 | W2 - W1])."""
import copy
import types

import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


def test_graph_feature_diff_mode(cuda):
    import oracle
    from dgx import synth
    from models.dgcnn import get_graph_feature
    x = torch.from_numpy(synth.cube_clouds(2, 300, 6)).permute(0, 2, 1).contiguous()
    idx = oracle.knn(x, 16)
    nbr = oracle.graph_feature(x.numpy(), idx, knn_only=True)             # (B,N,k,C)
    ctr = np.broadcast_to(x.numpy().transpose(0, 2, 1)[:, :, None, :], nbr.shape)
    ref = np.concatenate([nbr - ctr, ctr], axis=3).transpose(0, 3, 1, 2)
    xd = x.to(cuda).requires_grad_(True)
    out = get_graph_feature(xd, k=16, mode="diff")
    np.testing.assert_array_equal(out.detach().cpu().numpy(), ref)
    g = torch.randn_like(out)
    out.backward(g)
    xc = x.clone().requires_grad_(True)
    get_graph_feature(xc, k=16, mode="diff").backward(g.cpu())   # host path: torch autograd
    assert rel_err(xd.grad.cpu(), xc.grad) < 1e-6


def _reference_diff(m, x):
    """DGCNN with the paper's edge feature in stock PyTorch modules (fp32)."""
    from models.dgcnn import get_graph_feature
    h, outs = x, []
    for blk in m.edge_blocks():
        h = blk(get_graph_feature(h, m.k, mode="diff")).max(dim=-1)[0]
        outs.append(h)
    return m.conv5(torch.cat(outs, 1).unsqueeze(-1)).squeeze(-1)


def test_dgcnn_diff_mode_fp32(cuda):
    from dgx import synth
    torch.manual_seed(4)
    base = DGCNN_diff()
    x = torch.from_numpy(synth.cube_clouds(2, 512, 3)).to(cuda).permute(0, 2, 1)
    ma, mb = copy.deepcopy(base).to(cuda).train(), copy.deepcopy(base).to(cuda).train()
    ya = ma(x)
    yb = _reference_diff(mb, x)
    assert rel_err(ya.detach().cpu(), yb.detach().cpu()) < 1e-4
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    for (n, pa), pb in zip(ma.named_parameters(), mb.parameters()):
        assert rel_err(pa.grad.cpu(), pb.grad.cpu()) < 1e-3, n


def DGCNN_diff():
    from models.dgcnn import DGCNN
    return DGCNN(types.SimpleNamespace(emb_dim=256, k=16, edge_mode="diff"))


def test_dgcnn_diff_mode_is_reparameterised_cat(cuda, monkeypatch):
    """edge_mode "diff" with weights W equals edge_mode "cat" with [W1 | W2 - W1]
    bit for bit (forward), in both precision modes and through the C++ op."""
    from dgx import precision as prec
    from dgx import synth
    from models.dgcnn import DGCNN, _diff_weight
    torch.manual_seed(7)
    md = DGCNN_diff().to(cuda).train()
    mc = DGCNN(types.SimpleNamespace(emb_dim=256, k=16)).to(cuda).train()
    mc.load_state_dict(md.state_dict())
    with torch.no_grad():
        for bd, bc in zip(md.edge_blocks(), mc.edge_blocks()):
            bc[0].weight.copy_(_diff_weight(bd[0].weight))
    x = torch.from_numpy(synth.cube_clouds(2, 512, 5)).to(cuda).permute(0, 2, 1)
    for mode in ("fp32", "bf16"):
        prec.set(mode)
        try:
            assert torch.equal(md(x), mc(x)), mode
        finally:
            prec.set("fp32")
