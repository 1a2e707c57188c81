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
    """Output vs the stock-module restatement (fp32), and every parameter
    gradient vs the fp64 oracle routed by the engine's own decisions (neighbour
    sets, max slots, LeakyReLU signs) — the bar of test_edgeconv_gpu's
    test_dgcnn_train_routed, which a plain fp32-vs-fp32 comparison cannot hold:
    near-tied maxima route a gradient to different edges in two fp32 orders."""
    from dgx import synth
    from models.dgcnn import _diff_weight
    from oracle import reference as R
    from conftest import validate_dgcnn_decisions
    from test_edgeconv_gpu import ROUTED_GRAD_TOL, Capture
    torch.manual_seed(4)
    base = DGCNN_diff()
    init = {n: t.detach().clone() for n, t in base.state_dict().items()}
    x = torch.from_numpy(synth.cube_clouds(2, 512, 3)).to(cuda).permute(0, 2, 1)
    ma, mb = copy.deepcopy(base).to(cuda).train(), copy.deepcopy(base).to(cuda).train()
    with Capture() as cap:
        ya = ma(x)
    yb = _reference_diff(mb, x)
    assert rel_err(ya.detach().cpu(), yb.detach().cpu()) < 1e-4
    g = torch.randn_like(ya)
    ya.backward(g)
    # every block's neighbour set, max slot and LeakyReLU sign against the
    # reference's rules, on the equivalent (x_j, x_i) weights [W1 | W2 - W1]
    init_cat = dict(init)
    for i in range(1, 5):
        init_cat[f"conv{i}.0.weight"] = _diff_weight(init[f"conv{i}.0.weight"])
    print("decision check (gap, flip):", validate_dgcnn_decisions(cap, x, 16, init_cat))
    decisions = [tuple(t for t in cap[("fwd", l)]) for l in range(4)]
    p64 = {n: t.to(cuda).double() if t.is_floating_point() else t.to(cuda) for n, t in init.items()}
    for n, t in p64.items():
        if t.is_floating_point() and "running" not in n:
            t.requires_grad_(True)
    routed = dict(p64)
    for i in range(1, 5):
        routed[f"conv{i}.0.weight"] = _diff_weight(p64[f"conv{i}.0.weight"])
    ref = R.dgcnn_routed(x.double(), routed, [(i.long(), a, z) for (i, a, z) in decisions], ya.detach() > 0)
    assert rel_err(ya.detach().cpu(), ref.detach().cpu()) < 1e-4
    ref.backward(g.double())
    for n, p in ma.named_parameters():
        assert rel_err(p.grad.cpu(), p64[n].grad.cpu()) < ROUTED_GRAD_TOL, n


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
