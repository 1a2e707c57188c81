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


def _hog_agreement(got, ref):
    """(fraction of points bit-identical, fraction within HOG_TOL per point)."""
    exact = (got == ref).all(axis=-1)
    close = np.abs(got - ref).max(axis=-1) <= HOG_TOL
    return exact.mean(), close.mean()


# f1 tolerances. The reference runs the HOG votes with torch's kernels on the
# device it moved v and s to (model_partseg.py:42-47).
# * GPU votes (Net.forward's call on a GPU cloud, and any call without
#   use_cpu): the engine reproduces torch's HIP kernels op for op (ocml acosf /
#   atanf, reciprocal-multiply scalar division, the reduce kernel's sum and
#   norm order, GPU mean): EVERY point within HOG_TOL of the oracle running the
#   reference's op sequence on the GPU — every bin equal, no allowance.
# * host votes (use_cpu=True, the golden fixture): torch's CPU acos / atan are
#   glibc's scalar acosf (on the strided zenith input) and SLEEF's vectorised
#   atanf_u10 on chunks whose boundaries follow the host's thread split; the
#   engine rounds the fp64 function instead, so a point whose angle lands
#   within an ulp of an integer degree can take the neighbouring cell (one
#   whole vote): up to HOST_ALLOW of the points may differ.
HOG_TOL = 1e-6
HOST_ALLOW = 0.995


@pytest.mark.gpu
def test_hog_golden(golden, cuda):
    """The engine with host semantics (every stage as torch's CPU kernels)
    against the reference's own CPU run (tests/golden/partseg_small.npz)."""
    from dgx.hog import hog_1x1
    from models.dgcnn import knn
    g = golden("partseg_small.npz")
    x = torch.from_numpy(g["x"]).to(cuda)
    hog = hog_1x1(x, knn(x, 10), mean_device=False, votes_device=False)
    assert hog.is_cuda
    hog = hog.cpu().numpy()
    ref = g["hog"]
    assert hog.shape == ref.shape
    exact, close = _hog_agreement(hog, ref)
    assert exact >= HOST_ALLOW and close >= HOST_ALLOW, (exact, close)


def _oracle_semantics(x, idx, mean_dev, votes_dev, cuda):
    """The oracle's op sequence on the devices of each stage."""
    from oracle.hog import hog_1x1 as ref_hog
    xs = x.to(cuda) if mean_dev else x.cpu()
    return ref_hog(xs, idx.to(xs.device), cuda if votes_dev else "cpu").cpu().numpy()


SEMANTICS = [(True, True), (False, True), (True, False), (False, False)]


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,k", [(4, 1024, 20), (2, 2048, 40), (3, 500, 5), (2, 256, 64), (2, 777, 23)])
@pytest.mark.parametrize("sem", SEMANTICS, ids=lambda s: f"mean{'GPU' if s[0] else 'CPU'}_votes{'GPU' if s[1] else 'CPU'}")
def test_hog_device_vs_oracle(cuda, B, N, k, sem):
    """dgx_hog_1x1_sem_f32 vs the oracle running the reference's op sequence
    with each stage on the device the semantics name (mean: x's device; votes:
    where v and s were moved), on the same engine kNN ids. GPU votes: every
    point within 1e-6 (every bin equal); host votes: HOST_ALLOW."""
    from dgx.hog import hog_1x1
    from models.dgcnn import knn
    gen = torch.Generator().manual_seed(B * 1000 + k)
    x = torch.rand((B, 3, N), generator=gen) * 2 - 1
    xd = x.to(cuda)
    idx = knn(xd, k)
    got = hog_1x1(xd, idx, mean_device=sem[0], votes_device=sem[1]).cpu().numpy()
    ref = _oracle_semantics(x, idx, sem[0], sem[1], cuda)
    exact, close = _hog_agreement(got, ref)
    print(f"sem {sem}: exact {exact:.6f} close {close:.6f}")
    if sem[1]:
        assert close == 1.0, (exact, close)
    else:
        assert exact >= HOST_ALLOW and close >= HOST_ALLOW, (exact, close)


@pytest.mark.gpu
def test_hog_degenerate_neighbourhoods(cuda):
    """Repeated points: zero-spread neighbourhoods (SVD of a zero matrix) and
    collinear ones take dgesdd's exact-zero branches (GPU semantics, the
    reference's default path)."""
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
    ref = _oracle_semantics(x, idx, True, True, cuda)
    assert (np.isfinite(got) == np.isfinite(ref)).all()
    exact, close = _hog_agreement(np.nan_to_num(got), np.nan_to_num(ref))
    assert close == 1.0, (exact, close)


@pytest.mark.gpu
def test_hog_k_range(cuda):
    """The device HOG's k range is explicit: 5 and 64 run, 4 and 65 raise a clear
    NotImplementedError naming the range (not a bare C status code)."""
    from dgx.hog import HOG_K_MAX, HOG_K_MIN
    from models.model_partseg import compute_hog_1x1
    x = torch.rand((1, 3, 128), device=cuda)
    for k in (HOG_K_MIN, HOG_K_MAX):
        assert compute_hog_1x1(x, k).shape == (1, 128, 18)
    for k in (HOG_K_MIN - 1, HOG_K_MAX + 1):
        with pytest.raises(NotImplementedError, match="k <= 64"):
            compute_hog_1x1(x, k)


@pytest.mark.gpu
def test_hog_use_cpu_places_output(cuda, monkeypatch):
    """compute_hog_1x1's devices follow the reference's (model_partseg.py:32,
    42-47, 66-73): a GPU cloud with use_cpu=True takes the GPU mean and host
    votes and returns a host histogram; a host cloud without use_cpu takes
    the host mean and GPU votes and returns a GPU histogram — each equal to
    the oracle run with the same placement."""
    from models.dgcnn import knn
    from models.model_partseg import compute_hog_1x1
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    x = torch.rand((2, 3, 128), device=cuda)
    idx = knn(x, 8)
    h = compute_hog_1x1(x, 8, use_cpu=True)
    assert h.device.type == "cpu"
    exact, close = _hog_agreement(h.numpy(), _oracle_semantics(x, idx, True, False, cuda))
    assert exact >= HOST_ALLOW and close >= HOST_ALLOW, (exact, close)
    hc = compute_hog_1x1(x.cpu(), 8)
    assert hc.device.type == "cuda"
    exact, close = _hog_agreement(hc.cpu().numpy(), _oracle_semantics(x, idx, False, True, cuda))
    assert close == 1.0, (exact, close)
    # LOCAL_RANK moves the votes to the GPU even with use_cpu (model_partseg.py:42-44)
    monkeypatch.setenv("LOCAL_RANK", "0")
    assert compute_hog_1x1(x, 8, use_cpu=False).is_cuda


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


# Net at the partseg geometry (BASELINE cfg4: emb 512, k 40, N 2048; B 2 of the
# per-GPU shard), train mode, dropout 0, against the reference's forward over
# stock fp64 modules. The same forward over stock modules in the engine run's
# own precision (fp32, or fp32 weights under fp16 autocast as
# main_partseg_dist.py:253 runs it) measures how far the reference path itself
# lands from fp64 at that precision: this randomly initialised Net's
# gradients are ill-conditioned (BatchNorm over 4096 points, LeakyReLU kinks in
# the stock layers, near-zero gradients of cancelled parameters), stock fp32
# PyTorch is ~1e-2 off fp64 on several of them (tools/net_cfg4_probe.py). The
# engine must match fp64 as closely as the reference path does: per tensor
# err(engine) <= max(FLOOR, RATIO * err(stock)), output within the north
# star's 1e-3 (fp32) / AMP_TOL (fp16). Tensors whose true gradient is ~0
# (attention.out_proj.bias: a BatchNorm in the head cancels any per-channel
# constant) are measured against the model-wide gradient scale.
AMP_TOL = 2e-2
RATIO = 1.5
# precision "fp32_split" (opt-in): conv5's GEMMs and blocks 2-4's weight / input
# gradients as 3-pass split bf16 (~2^-16 relative per product instead of fp32's
# 2^-24) and dz packed with its slot (18 significant bits), which the
# ill-conditioned gradients above amplify to ~2x stock fp32's error on a few
# EdgeConv weights (r06u: conv4.0.weight 9.6e-3 vs stock 4.8e-3; 6.0e-3 vs
# 6.0e-3 worst with exact products). The exact default is held to RATIO.
RATIO_SPLIT = 3.0
# amp: under fp16 autocast the engine's DGCNN GEMMs run split-bf16 (16
# significant bits per operand, dgx.precision.effective) and its edge MLP exact
# fp32, never narrower than the stock layers' fp16 (11 bits): the engine's
# share of the error stays below the stock fp16 step's.
RATIO_AMP = 2.0
# The engine's own parameters (emb_nn, the edge MLP's conv1 / conv2 / bn1 /
# bn2) are held to the mode's ratio above. The stock layers' parameters
# (transformer, attention projections, MLPs, the PositionEmbedding transform)
# are computed by torch's kernels in BOTH runs, fed differently rounded inputs
# (and, in fp32 / fp32_split, the engine attention's split-bf16 planes, ~2^-16
# per product); their error against fp64 moves by up to ~2x between two such
# runs of the same code (r09b / r09i: head.nn.5.bias 2.0x once, passing <1.5x
# the run before; amp: pos_mlp.0.transform.bias 2.03x): RATIO_STOCK.
RATIO_STOCK = 2.5
ENGINE_OWNED = ("emb_nn.", "pos_mlp.0.conv1.", "pos_mlp.0.conv2.", "pos_mlp.0.bn1.", "pos_mlp.0.bn2.")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fp32", "fp32_split", "amp"])
def test_net_cfg4_routed(cuda, mode, monkeypatch):
    """Net train step at cfg4 geometry against the reference's forward over
    stock fp64 modules (oracle.partseg.net_routed) on the same neighbours:
    every EdgeConv kNN / max slot / sign, the edge stage's kNN / conv2 slot /
    sign, PositionEmbedding's max over points and the HOG are validated, then
    the output and EVERY parameter gradient are compared. fp32: the default
    precision (exact fp32 GEMM products); fp32_split: the opt-in split-bf16
    GEMMs; amp: fp16 autocast as main_partseg_dist.py:253 trains (the
    engine's GEMMs then run split-bf16)."""
    import dgx.edgeconv as E
    from dgx import precision as prec
    amp = mode == "amp"
    monkeypatch.setattr(prec, "_mode", "fp32_split" if mode == "fp32_split" else "fp32")
    ratio = {"fp32": RATIO, "fp32_split": RATIO_SPLIT, "amp": RATIO_AMP}[mode]
    import oracle
    from conftest import edge_mlp_decisions, validate_dgcnn_decisions
    from dgx import synth
    from models.model_partseg import Net, compute_hog_1x1
    from oracle.hog import hog_1x1 as ref_hog
    from oracle.partseg import net_routed, stock_copy
    B, N, k, emb = 2, 2048, 40, 512
    args = types.SimpleNamespace(k=k, emb_dim=emb, n_heads=4, n_blocks=1, ff_dims=512, dropout=0.0, nclasses=50)
    # deterministic MIOpen solvers for the stock layers of both runs, so the
    # engine-vs-stock error ratio below is a property of the code, not of the
    # solver each run happened to pick
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    monkeypatch.setattr(torch.backends.cudnn, "benchmark", False)
    torch.manual_seed(17)
    net = Net(args)
    net64 = stock_copy(net).double().to(cuda).train()
    net32 = stock_copy(net).to(cuda).train()
    init_emb = {n: t.detach().clone() for n, t in net.emb_nn.state_dict().items()}
    net = net.to(cuda).train()
    pts = synth.cube_clouds(B, N, 170)
    src = torch.from_numpy(pts).to(cuda).permute(0, 2, 1).contiguous()
    lbl = torch.nn.functional.one_hot(torch.tensor([3, 11]), 16).float().to(cuda)
    gout = torch.from_numpy(synth.uniform(171, (B, 50, N)) - 0.5).float().to(cuda)
    seen = {}
    hooks = [net.emb_nn.register_forward_hook(lambda m, i, o: seen.__setitem__("emb", o.detach())),
             net.pos_mlp[0].conv3.register_forward_hook(lambda m, i, o: seen.__setitem__("t3", o.detach()))]
    E.set_debug_capture({})
    try:
        with torch.autocast("cuda", dtype=torch.float16, enabled=amp):
            out = net(src, lbl)
        out.float().backward(gout)
        cap = E.debug_capture()
    finally:
        E.set_debug_capture(None)
        for h in hooks:
            h.remove()
    # decisions: DGCNN blocks, edge stage, max over points, HOG (the forward
    # EdgeConv GEMMs are exact fp32 in every mode but bf16, so the decisions
    # are checked against the fp32 recomputation)
    dec = validate_dgcnn_decisions(cap, src, k, init_emb, bf16=False)
    dgcnn_dec = [(i.long(), a, z) for (i, a, z) in (cap[("fwd", l)] for l in range(4))]
    zpos1, arg2, zpos2, edec = edge_mlp_decisions(cap, B, N, k, net.pos_mlp[0].conv2[0].weight)
    eidx = cap["emlp"]["idx"].view(B, N, k).long()
    np.testing.assert_array_equal(eidx.cpu().numpy(), oracle.knn(src.cpu(), k))
    argmax_n = seen["t3"].max(dim=-1)[1]
    # the HOG the engine fed grads_emb (model_partseg.py:179) vs the reference's op
    # sequence on the GPU (Net.forward's path for a GPU cloud): every point
    net_hog = compute_hog_1x1(src, k)
    hog = ref_hog(src, torch.from_numpy(oracle.knn(src.cpu(), k)).to(cuda), cuda).cpu()
    exact, close = _hog_agreement(net_hog.cpu().numpy(), hog.numpy())
    assert close == 1.0, (exact, close)
    runs = {}
    for name, m, dt in (("f64", net64, torch.float64), ("stock", net32, torch.float32)):
        with torch.autocast("cuda", dtype=torch.float16, enabled=amp and name == "stock"):
            r, t3 = net_routed(m, src.to(dt), lbl.to(dt), dgcnn_dec, seen["emb"] > 0, (eidx, zpos1, arg2, zpos2),
                               net_hog.to(dt), argmax_n)
        r.float().backward(gout) if name == "stock" else r.backward(gout.double())
        runs[name] = (r.detach(), dict(m.named_parameters()), t3.detach())
    t3 = runs["f64"][2]
    gap_n = float((t3.max(dim=-1)[0] - torch.gather(t3, 2, argmax_n.unsqueeze(-1)).squeeze(-1)).max()
                  / t3.abs().max())
    # under autocast the stock conv3 before the max over points runs fp16 (unit
    # roundoff 2^-11): a near-tied max may pick a point whose fp64 value trails
    # the maximum by a few fp16 ulps of the scale
    assert gap_n <= (2e-3 if amp else 1e-5), ("max over points", gap_n)
    ref = runs["f64"][0].cpu()
    e_out = rel_err(out.detach().float().cpu(), ref)
    assert e_out < (AMP_TOL if amp else TOL), ("out", e_out)
    floor = AMP_TOL if amp else TOL
    g64 = runs["f64"][1]
    gscale = max(float(p.grad.abs().max()) for p in g64.values())

    def err(got, want):
        want = want.cpu().double()
        den = max(float(want.abs().max()), 1e-3 * gscale)
        return float((got.cpu().double() - want).abs().max()) / den
    rows = []
    for n, p in net.named_parameters():
        rows.append((n, err(p.grad, g64[n].grad), err(runs["stock"][1][n].grad, g64[n].grad)))
    rows.sort(key=lambda r: -r[1] / max(floor, ratio * r[2]))
    print(f"Net cfg4 {mode}: decisions {dec} edge {edec} maxN gap {gap_n:.1e}; out {e_out:.1e}; "
          "worst (engine, stock):", [(n, f"{e:.1e}", f"{e2:.1e}") for n, e, e2 in rows[:6]])
    for n, e, e2 in rows:
        r = ratio if n.startswith(ENGINE_OWNED) else max(ratio, RATIO_STOCK)
        assert e <= max(floor, r * e2), (n, e, e2)


@pytest.mark.gpu
def test_net_knn_computed_once(cuda, monkeypatch):
    """Net.forward's three kNN of the input cloud (model_partseg.py:177, 179,
    183) run as ONE selection launch (dgx.ops.knn_cache), and the step is
    bit-identical to the one that computes them three times."""
    import contextlib
    import models.model_partseg as MP
    from dgx import ops, synth
    args = types.SimpleNamespace(k=20, emb_dim=64, n_heads=4, n_blocks=1, ff_dims=128, dropout=0.0, nclasses=50)
    # the stock Conv1d layers of Net (grads_emb, head) run on MIOpen, whose
    # weight-gradient solvers may accumulate in a run-dependent order: pin
    # deterministic solvers so the comparison isolates the engine path
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    monkeypatch.setattr(torch.backends.cudnn, "benchmark", False)
    torch.manual_seed(3)
    net = MP.Net(args).to(cuda).train()
    init = {n: t.clone() for n, t in net.state_dict().items()}
    src = torch.from_numpy(synth.cube_clouds(2, 512, 12)).to(cuda).permute(0, 2, 1).contiguous()
    lbl = torch.nn.functional.one_hot(torch.tensor([3, 7]), 16).float().to(cuda)

    def step():
        net.load_state_dict(init)
        net.zero_grad(set_to_none=True)
        timing = []
        ops.set_knn_timing(timing)
        try:
            out = net(src, lbl)
        finally:
            ops.set_knn_timing(None)
        out.square().mean().backward()
        return out.detach(), {n: p.grad.clone() for n, p in net.named_parameters()}, \
            sum(1 for t in timing if t[3][1] == 3)
    out1, g1, n1 = step()
    monkeypatch.setattr(MP, "knn_cache", contextlib.nullcontext)
    out3, g3, n3 = step()
    assert (n1, n3) == (1, 3)
    assert torch.equal(out1, out3)
    for n in g1:
        assert torch.equal(g1[n], g3[n]), n
