"""a7/a9/f1 parity: compute_hog_1x1 (engine kNN + device HOG) and the partseg
Net callers (reference models/model_partseg.py:15-194) against
tests/golden/partseg_small.npz and the oracle's HOG restatement."""
import types

import numpy as np
import pytest
import torch

from conftest import rel_err

TOL = 1e-3
BIG = ("pos_mlp.0.conv3.0.weight", "pos_mlp.0.linear.0.weight")
ARGS = types.SimpleNamespace(emb_dim=64, k=10, n_heads=4, n_blocks=1, ff_dims=128, dropout=0.0, nclasses=50)


def _big_init(i, shape):
    # same deterministic init make_goldens.py:partseg_big_init applied to the reference
    from dgx import synth
    return ((synth.uniform(63 + i, shape) - 0.5) * (2.0 / np.sqrt(shape[1]))).astype(np.float32)


def _net(g):
    from models.model_partseg import Net
    net = Net(ARGS)
    state = {k[5:]: torch.from_numpy(np.asarray(g[k])) for k in g.files if k.startswith("init.")}
    for i, n in enumerate(BIG):
        state[n] = torch.from_numpy(_big_init(i, tuple(net.get_parameter(n).shape)))
    missing, unexpected = net.load_state_dict(state, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    return net


def test_net_state_dict_matches_reference(golden):
    """Every reference key (incl. PositionEmbedding aliases) loads, shapes agree."""
    g = golden("partseg_small.npz")
    from models.model_partseg import Net
    sd = Net(ARGS).state_dict()
    ref_keys = {k[5:] for k in g.files if k.startswith("init.")} | set(BIG)
    assert set(sd.keys()) == ref_keys
    for k in ref_keys & set(sd.keys()):
        if "init." + k in g.files:
            assert tuple(sd[k].shape) == g["init." + k].shape, k


def test_product_rejects_cpu_tensors():
    """The engine has no CPU fallback: a CPU cloud fails loudly at the kNN."""
    from models.model_partseg import compute_hog_1x1
    with pytest.raises(RuntimeError):
        compute_hog_1x1(torch.zeros(1, 3, 32), 4, use_cpu=True)


def _hog_agreement(got, ref):
    """(fraction of points bit-identical, fraction within HOG_TOL per point)."""
    exact = (got == ref).all(axis=-1)
    close = np.abs(got - ref).max(axis=-1) <= HOG_TOL
    return exact.mean(), close.mean()


# f1 tolerance: the device HOG follows the reference op by op (torch CPU sum
# order, fp64 SVD as numpy's dgesdd, fp32 angle ops), so points agree bit-for-bit
# except where an fp32 acos/atan differs from the host libm's in the last ulp
# right at an integer degree (.int() then moves the vote to the next cell).
# Such a point differs by up to a whole vote; every other point is exact.
HOG_TOL = 1e-6


@pytest.mark.gpu
def test_hog_golden(golden, cuda):
    from models.model_partseg import compute_hog_1x1
    g = golden("partseg_small.npz")
    x = torch.from_numpy(g["x"]).to(cuda)
    hog = compute_hog_1x1(x, 10)
    assert hog.is_cuda
    hog = hog.cpu().numpy()
    ref = g["hog"]
    assert hog.shape == ref.shape
    exact, close = _hog_agreement(hog, ref)
    assert exact >= 0.995 and close >= 0.995, (exact, close)


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,k", [(4, 1024, 20), (2, 2048, 40), (3, 500, 5), (2, 256, 64)])
def test_hog_device_vs_oracle(cuda, B, N, k):
    """dgx_hog_1x1_f32 vs the oracle restatement on the same engine kNN ids."""
    from oracle.hog import hog_1x1 as ref_hog
    from dgx.hog import hog_1x1
    from models.dgcnn import knn
    gen = torch.Generator().manual_seed(B * 1000 + k)
    x = torch.rand((B, 3, N), generator=gen) * 2 - 1
    xd = x.to(cuda)
    idx = knn(xd, k)
    got = hog_1x1(xd, idx).cpu().numpy()
    ref = ref_hog(x, idx.cpu()).numpy()
    exact, close = _hog_agreement(got, ref)
    assert exact >= 0.995 and close >= 0.995, (exact, close)


@pytest.mark.gpu
def test_hog_degenerate_neighbourhoods(cuda):
    """Repeated points: zero-spread neighbourhoods (SVD of a zero matrix) and
    collinear ones take dgesdd's exact-zero branches."""
    from oracle.hog import hog_1x1 as ref_hog
    from dgx.hog import hog_1x1
    from models.dgcnn import knn
    N, k = 256, 10
    base = torch.rand((1, 3, 16), generator=torch.Generator().manual_seed(5))
    x = base.repeat_interleave(N // 16, dim=2).contiguous()      # 16 copies of each point
    line = torch.linspace(-1, 1, N).view(1, 1, N) * torch.tensor([1.0, 2.0, -0.5]).view(1, 3, 1)
    x = torch.cat([x, line], dim=0).contiguous()
    xd = x.to(cuda)
    idx = knn(xd, k)
    got = hog_1x1(xd, idx).cpu().numpy()
    ref = ref_hog(x, idx.cpu()).numpy()
    assert np.isfinite(got).all() == np.isfinite(ref).all()
    exact, close = _hog_agreement(np.nan_to_num(got), np.nan_to_num(ref))
    assert close >= 0.99, (exact, close)


@pytest.mark.gpu
def test_hog_use_cpu_places_output(cuda, monkeypatch):
    from models.model_partseg import compute_hog_1x1
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    x = torch.rand((2, 3, 128), device=cuda)
    assert compute_hog_1x1(x, 8, use_cpu=True).device.type == "cpu"
    with pytest.raises(RuntimeError):
        compute_hog_1x1(x.cpu(), 8)


@pytest.mark.gpu
def test_hog_knn_is_engine_knn(golden, cuda):
    """The a7 row proper: the kNN compute_hog_1x1 uses is the engine's, bit-exact."""
    import oracle
    from models.dgcnn import knn
    g = golden("partseg_small.npz")
    x = torch.from_numpy(g["x"]).to(cuda)
    idx = knn(x, 10)
    assert idx.dtype == torch.int64 and idx.is_cuda
    ref = oracle.knn(g["x"], 10)
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)


@pytest.mark.gpu
def test_net_golden(golden, cuda):
    g = golden("partseg_small.npz")
    net = _net(g).to(cuda).train()
    x = torch.from_numpy(g["x"]).to(cuda)
    lbl = torch.from_numpy(g["lbl"]).to(cuda)
    y = net(x, lbl)
    assert tuple(y.shape) == g["out"].shape
    assert rel_err(y.detach().cpu(), g["out"]) < TOL
    y.backward(torch.from_numpy(g["gout"]).to(cuda))
    # gradients pass through max_k / LeakyReLU kinks: all but
    # a few elements per tensor agree to 1e-3 of the tensor's scale. Tensors
    # whose true gradient is ~0 (e.g. attention.out_proj.bias: a BatchNorm in
    # the head cancels any per-channel constant) use the model-wide scale.
    from dgx import synth
    gscale = max(np.abs(g[k]).max() for k in g.files if k.startswith("grad."))
    for n, p in net.named_parameters():
        if "grad." + n in g.files:
            ref = g["grad." + n]
            got = p.grad.cpu().numpy()
            close = (np.abs(got - ref) <= TOL * max(np.abs(ref).max(), 1e-3 * gscale)).mean()
            assert close >= 0.98, (n, close)
        elif "gradproj." + n in g.files:
            i = BIG.index(n)
            r = synth.uniform(70 + i, tuple(p.shape)) - 0.5
            proj = g["gradproj." + n]
            got = p.grad.cpu().double().numpy()
            assert abs(np.linalg.norm(got) - proj[1]) <= 2e-2 * proj[1], n
            assert abs((got * r).sum() - proj[0]) <= 2e-2 * proj[1] * np.sqrt(r.size) * 0.3, n


def test_hog_restatement_matches_reference_cpu(golden):
    """The oracle's HOG restatement (oracle/hog.py), fed the oracle's kNN,
    reproduces the reference's CPU run bit-for-bit: this pins the checker the
    device HOG is compared with."""
    import oracle
    from oracle.hog import hog_1x1
    g = golden("partseg_small.npz")
    idx = torch.from_numpy(oracle.knn(g["x"], 10))
    hog = hog_1x1(torch.from_numpy(g["x"]), idx).numpy()
    np.testing.assert_array_equal(hog, g["hog"])
