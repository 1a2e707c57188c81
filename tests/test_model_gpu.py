"""model.DGCNN_cls / DGCNN_semseg (engine-backed; architecture unpinned by the
reference, see model.py) against the same layer list run as stock PyTorch ops
in float64 on the same weights and the same neighbour sets (the engine's kNN
is bit-exact with the reference's: test_knn_gpu.py)."""
import copy
import types

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
from conftest import rel_err
from oracle import reference as R

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _capture():
    import dgx.edgeconv as E
    E.set_debug_capture({})
    return E


def _cls_reference(m, x, idxs):
    B = x.shape[0]
    h, feats = x, []
    for i, conv in enumerate((m.conv1, m.conv2, m.conv3, m.conv4)):
        h = conv(R.graph_feature(h, idx=idxs[i])).max(dim=-1)[0]
        feats.append(h)
    h = m.conv5(torch.cat(feats, dim=1))
    h = torch.cat((F.adaptive_max_pool1d(h, 1).view(B, -1), F.adaptive_avg_pool1d(h, 1).view(B, -1)), 1)
    h = m.dp1(F.leaky_relu(m.bn6(m.linear1(h)), 0.2))
    h = m.dp2(F.leaky_relu(m.bn7(m.linear2(h)), 0.2))
    return m.linear3(h)


@pytest.mark.parametrize("train", [True, False])
def test_dgcnn_cls_matches_stock_ops(cuda, train):
    from dgx import synth
    from model import DGCNN_cls
    torch.manual_seed(21)
    args = types.SimpleNamespace(k=20, emb_dims=256, dropout=0.0)
    m = DGCNN_cls(args)
    ref_m = copy.deepcopy(m).double().to(cuda)
    m = m.to(cuda)
    m.train(train)
    ref_m.train(train)
    if not train:
        with torch.no_grad():  # non-trivial running statistics
            for mod in (m, ref_m):
                for n, b in mod.named_buffers():
                    if n.endswith("running_var"):
                        b.copy_(torch.linspace(0.5, 2.0, b.numel(), device=cuda))
    pts = synth.cube_clouds(8, 1024, 77)
    x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
    E = _capture()
    try:
        y = m(x)
        dec = E.debug_capture()
    finally:
        E.set_debug_capture(None)
    if train:
        idxs = [dec[("fwd", l)][0].long() for l in range(4)]
    else:  # eval: the fused inference path records nothing; the neighbours come from the oracle
        idxs = None
    with torch.no_grad():
        if idxs is None:
            xs = torch.from_numpy(pts).permute(0, 2, 1)
            idxs = [torch.as_tensor(oracle.knn(xs, 20)).long().to(cuda)] + [None] * 3
            ref = None
            h, feats = xs.double().to(cuda), []
            for i, conv in enumerate((ref_m.conv1, ref_m.conv2, ref_m.conv3, ref_m.conv4)):
                idx = idxs[i] if i == 0 else torch.as_tensor(
                    oracle.knn(h.float().cpu().contiguous(), 20)).long().to(cuda)
                h = conv(R.graph_feature(h, idx=idx)).max(dim=-1)[0]
                feats.append(h)
            hh = ref_m.conv5(torch.cat(feats, 1))
            B = hh.shape[0]
            hh = torch.cat((F.adaptive_max_pool1d(hh, 1).view(B, -1), F.adaptive_avg_pool1d(hh, 1).view(B, -1)), 1)
            hh = F.leaky_relu(ref_m.bn6(ref_m.linear1(hh)), 0.2)
            ref = ref_m.linear3(F.leaky_relu(ref_m.bn7(ref_m.linear2(hh)), 0.2))
        else:
            ref = _cls_reference(ref_m, torch.from_numpy(pts).to(cuda).double().permute(0, 2, 1), idxs)
    assert y.shape == (8, 40)
    assert rel_err(y.detach().cpu(), ref.cpu()) < TOL
    if train:
        y.square().sum().backward()
        assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


def test_dgcnn_semseg_stages_match_stock_ops(cuda):
    """Each stage of DGCNN_semseg (2-conv blocks with the first graph on xyz
    channels 6:9, the 1-conv block, conv6 + global max, the per-point head)
    equals the stock op sequence on the engine's own stage inputs."""
    from dgx import synth
    from dgx.edgeconv import edgeconv_stack_pair
    from dgx.edgemlp import edge_mlp2
    from model import DGCNN_semseg
    torch.manual_seed(22)
    args = types.SimpleNamespace(k=20, emb_dims=256, dropout=0.0)
    m = DGCNN_semseg(args).to(cuda).train()
    ref_m = copy.deepcopy(m).double()
    blk = synth.s3dis_blocks(2, 1024, seed=5)
    x = torch.from_numpy(blk).to(cuda).permute(0, 2, 1).contiguous()
    y = m(x)
    assert y.shape == (2, 13, 1024)
    with torch.no_grad():
        # stage by stage on the engine's own intermediate features
        x1 = edge_mlp2(x, 20, copy.deepcopy(m.conv1), copy.deepcopy(m.conv2), knn_src=x[:, 6:9])
        idx1 = torch.as_tensor(oracle.knn(x[:, 6:9].cpu(), 20)).long().to(cuda)
        r1 = ref_m.conv2(ref_m.conv1(R.graph_feature(x.double(), idx=idx1))).max(-1)[0]
        assert rel_err(x1.cpu(), r1.cpu()) < TOL
        x1c = x1.contiguous()
        x2 = edge_mlp2(x1c, 20, copy.deepcopy(m.conv3), copy.deepcopy(m.conv4))
        idx2 = torch.as_tensor(oracle.knn(x1c.cpu(), 20)).long().to(cuda)
        r2 = ref_m.conv4(ref_m.conv3(R.graph_feature(x1c.double(), idx=idx2))).max(-1)[0]
        assert rel_err(x2.cpu(), r2.cpu()) < TOL
        x2c = x2.contiguous()
        x3, _ = edgeconv_stack_pair(x2c, 20, [copy.deepcopy(m.conv5)])
        idx3 = torch.as_tensor(oracle.knn(x2c.cpu(), 20)).long().to(cuda)
        r3 = ref_m.conv5(R.graph_feature(x2c.double(), idx=idx3)).max(-1)[0]
        assert rel_err(x3.view(2, 1024, -1).permute(0, 2, 1).cpu(), r3.cpu()) < TOL
    y.square().mean().backward()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


@pytest.mark.parametrize("precision_mode", ["bf16", "fp32"])
def test_dgcnn_train_step_graph_replay_equals_eager(cuda, precision_mode):
    """bench.py times the N=1 train step as one HIP-graph replay (torch.cuda.CUDAGraph
    capture of fwd + bwd + SGD): every engine launch goes to the capture stream,
    nothing syncs the host, and one replay from a given state gives bit-for-bit
    the parameters and BN statistics of one eager step from that state."""
    from dgx import precision, synth
    from models.dgcnn import DGCNN
    torch.manual_seed(3)
    precision.set(precision_mode)
    try:
        m = DGCNN(types.SimpleNamespace(emb_dim=256, k=20)).to(cuda).train()
        init = copy.deepcopy(m.state_dict())
        opt = torch.optim.SGD(m.parameters(), lr=0.05)
        x = torch.from_numpy(synth.cube_clouds(4, 512, 1)).to(cuda).permute(0, 2, 1)
        gy = torch.from_numpy(synth.uniform(2, (4, 256, 512)) - 0.5).float().to(cuda)

        def step():
            opt.zero_grad(set_to_none=True)
            m(x).backward(gy)
            opt.step()

        side = torch.cuda.Stream(cuda)
        side.wait_stream(torch.cuda.current_stream(cuda))
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream(cuda).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(graph):
            m(x).backward(gy)
            opt.step()
        m.load_state_dict(init)  # in place: the captured buffers stay valid
        graph.replay()
        torch.cuda.synchronize()
        replayed = {n: t.clone() for n, t in m.state_dict().items()}
        m.load_state_dict(init)
        step()
        torch.cuda.synchronize()
        for n, t in m.state_dict().items():
            assert torch.equal(t, replayed[n]), n
    finally:
        precision.set("fp32")
