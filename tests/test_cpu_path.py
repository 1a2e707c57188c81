"""SURVEY §8(b) "CPU tensors -> CPU restatement path": the drop-in modules on
host tensors (dgx.cpu), against the reference's goldens — no GPU, no oracle
on the product side. BASELINE cfg1 (main_cls.py, B=4 on the host) runs the
same path: models.dgcnn / model.DGCNN_cls on CPU tensors."""
import types

import numpy as np
import pytest
import torch

from conftest import assert_knn_equivalent, load_golden, rel_err

KNN_CASES = ["c3", "c9", "c64", "c128", "c3k40", "c64k32", "c3n1000"]


def _cpu_view(pts, layout):
    t = torch.from_numpy(pts)
    return t.permute(0, 2, 1) if layout == "perm" else t.permute(0, 2, 1).contiguous()


@pytest.mark.parametrize("layout", ["bcn", "perm"])
@pytest.mark.parametrize("case", KNN_CASES)
def test_cpu_knn_matches_reference_golden(case, layout):
    """Bit-exact selected values and canonical indices on the host (the
    reference's own op sequence, stable top-k)."""
    from models.dgcnn import knn
    g = load_golden("knn_cases.npz")
    key = f"{case}_{layout}"
    idx = knn(_cpu_view(g[key + "_x"], layout), g[key + "_idx"].shape[-1])
    assert idx.dtype == torch.int64 and idx.device.type == "cpu"
    np.testing.assert_array_equal(idx.numpy(), g[key + "_idx"])


def test_cpu_knn_ties_golden():
    import oracle
    from models.dgcnn import knn
    g = load_golden("knn_cases.npz")
    x = _cpu_view(g["ties_perm_x"], "perm")
    idx = knn(x, 20).numpy()
    pd = oracle.pairwise(x)   # test-side checker: values of the chosen ids
    assert_knn_equivalent(idx, np.take_along_axis(pd, idx, 2), g["ties_perm_idx"], g["ties_perm_val"])


@pytest.mark.parametrize("which", ["xyz", "feat"])
def test_cpu_graph_feature_golden(which):
    from models.dgcnn import get_graph_feature
    g = load_golden("graph_feature.npz")
    x = torch.from_numpy(g[f"{which}_x"])
    k = g[f"{which}_idx"].shape[-1]
    np.testing.assert_array_equal(get_graph_feature(x, k).numpy(), g[f"{which}_cat"])
    np.testing.assert_array_equal(get_graph_feature(x, k, disp_only=True).numpy(), g[f"{which}_disp"])
    np.testing.assert_array_equal(get_graph_feature(x, k, knn_only=True).numpy(), g[f"{which}_knn"])


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_cpu_library_graph_feature_op(mode):
    """torch.ops.dgx.graph_feature on host tensors (CPU kernel + the op's
    autograd formula) equals the differentiable host restatement."""
    import dgx.library  # noqa: F401
    from dgx import cpu, synth
    x = torch.from_numpy(synth.cube_clouds(2, 96, 4)).permute(0, 2, 1).contiguous()
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    out, idx = torch.ops.dgx.graph_feature(xa, 10, mode)
    ref = cpu.graph_feature(xb, 10, knn_only=mode == 2, disp_only=mode == 1)
    assert torch.equal(out, ref) and idx.dtype == torch.int32
    go = torch.randn_like(out)
    out.backward(go)
    ref.backward(go)
    assert rel_err(xa.grad, xb.grad) < 1e-6
    assert torch.equal(torch.ops.dgx.knn(x, 10), cpu.knn(x, 10))


def _block(w, gamma, beta):
    co, c2 = w.shape[0], w.shape[1]
    blk = torch.nn.Sequential(torch.nn.Conv2d(c2, co, 1, bias=False), torch.nn.BatchNorm2d(co),
                              torch.nn.LeakyReLU(0.2, inplace=True))
    with torch.no_grad():
        blk[0].weight.copy_(torch.from_numpy(w))
        blk[1].weight.copy_(torch.from_numpy(gamma))
        blk[1].bias.copy_(torch.from_numpy(beta))
    return blk


def test_cpu_edgeconv_block_golden():
    from dgx.edgeconv import edgeconv_stack
    g = load_golden("edgeconv_block.npz")
    blk = _block(g["weight"], g["gamma"], g["beta"])
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    B, C, N = x.shape
    y = edgeconv_stack(x, int(g["k"]), [blk], True).view(B, N, -1).permute(0, 2, 1)
    assert rel_err(y.detach(), g["out"]) < 1e-3
    y.backward(torch.from_numpy(g["gout"]))
    for got, key in ((x.grad, "dx"), (blk[0].weight.grad, "dweight"), (blk[1].weight.grad, "dgamma"),
                     (blk[1].bias.grad, "dbeta")):
        assert rel_err(got, g[key]) < 1e-3, key
    assert rel_err(blk[1].running_mean, g["running_mean"]) < 1e-5
    assert rel_err(blk[1].running_var, g["running_var"]) < 1e-5


def test_cpu_dgcnn_train_golden():
    """DGCNN(emb 64, k 10) train step on host tensors against the reference's
    fp32 run: output at 1e-3, running statistics; gradients at the GPU test's
    unrouted bar (the fixture holds a LeakyReLU kink at |z| ~ 1e-7)."""
    from models.dgcnn import DGCNN
    g = load_golden("dgcnn_small.npz")
    m = DGCNN(types.SimpleNamespace(emb_dim=64, k=10))
    m.load_state_dict({n[5:]: torch.from_numpy(g[n]) for n in g.files if n.startswith("init.")})
    m.train()
    y = m(torch.from_numpy(g["x"]))
    assert y.device.type == "cpu" and rel_err(y.detach(), g["out"]) < 1e-3
    y.backward(torch.from_numpy(g["gout"]))
    for n, p in m.named_parameters():
        assert rel_err(p.grad, g["grad." + n]) < 5e-2, n
    for n, b in m.state_dict().items():
        if "running" in n:
            assert rel_err(b, g["after." + n]) < 1e-4, n


def test_cpu_position_embedding_golden():
    import hashlib
    from models.layers import PositionEmbedding
    g = load_golden("posemb_small.npz")
    torch.manual_seed(5)
    m = PositionEmbedding(types.SimpleNamespace(k=10))
    with torch.no_grad():
        m.transform.weight.normal_(0, 0.05)
    sha = hashlib.sha256(b"".join(v.detach().numpy().tobytes() for v in m.state_dict().values())).hexdigest()
    assert sha == str(g["init_sha256"])
    m.train()
    y = m(torch.from_numpy(g["x"]))
    assert rel_err(y.detach(), g["out"]) < 1e-3


def test_cpu_hog_golden():
    """compute_hog_1x1(use_cpu=True) on host tensors: the reference's host
    algorithm (numpy LAPACK SVD), equal to its golden histograms."""
    from models.model_partseg import compute_hog_1x1
    g = load_golden("partseg_small.npz")
    h = compute_hog_1x1(torch.from_numpy(g["x"]), 10, use_cpu=True)
    assert h.device.type == "cpu"
    np.testing.assert_allclose(h.numpy(), g["hog"], rtol=0, atol=1e-6)


def test_cpu_dgcnn_cls_cfg1_train_step():
    """BASELINE cfg1's plumbing: model.DGCNN_cls (main_cls.py:56) on a B=4,
    N=1024, k=20 host batch fed as main_cls.py:91 feeds it (a permuted view),
    one SGD step: finite loss and gradients, BN statistics updated."""
    from dgx import synth
    from model import DGCNN_cls
    from util import cal_loss
    torch.manual_seed(0)
    args = types.SimpleNamespace(k=20, emb_dims=1024, emb_dim=1024, dropout=0.5)
    m = DGCNN_cls(args).train()
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.from_numpy(synth.cube_clouds(4, 1024, 3)).permute(0, 2, 1)
    label = torch.tensor([1, 5, 7, 39])
    logits = m(x)
    loss = cal_loss(logits, label)
    loss.backward()
    opt.step()
    assert torch.isfinite(loss) and logits.shape == (4, 40)
    assert all(p.grad is None or torch.isfinite(p.grad).all() for p in m.parameters())


def test_cpu_net_golden(monkeypatch):
    """The partseg Net (reference model_partseg.py:142-194, emb 64, one
    transformer block, dropout 0) on host tensors against the reference's
    golden forward; as when the golden was made, the HOG histogram stays on
    the host (the reference's use_cpu=True, model_partseg.py:66-73)."""
    import models.model_partseg as MP
    from test_partseg import _net
    g = load_golden("partseg_small.npz")
    monkeypatch.setattr(MP, "_hist_device", lambda use_cpu: torch.device("cpu"))
    net = _net(g).train()
    y = net(torch.from_numpy(g["x"]), torch.from_numpy(g["lbl"]))
    assert y.device.type == "cpu" and tuple(y.shape) == g["out"].shape
    assert rel_err(y.detach(), g["out"]) < 1e-3
