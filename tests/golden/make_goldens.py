"""Generate tests/golden/*.npz from the REFERENCE itself (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py
It imports /root/reference/models (read-only; nothing is written there) and
records inputs, outputs and gradients of the hot path as data fixtures. The
reference's source never leaves the build container; only these vectors do.

Fixtures
  knn_cases.npz      reference knn (dgcnn.py:6-12) on synthetic clouds, C in
                     {3,9,64,128}, both memory layouts, plus a duplicate-point
                     tie set; indices in canonical order + selected pd values.
  graph_feature.npz  get_graph_feature (dgcnn.py:15-44), all three modes.
  edgeconv_block.npz one block: get_graph_feature -> conv/BN/LReLU -> max (train
                     BN, gamma with negative entries): out, dx, dW, dgamma,
                     dbeta, running stats.
  dgcnn_small.npz    DGCNN(emb=64) train-mode fwd + bwd on (2,3,128), k=10.
  posemb_small.npz   PositionEmbedding fwd + bwd on (2,3,128), k=10.
  partseg_small.npz  compute_hog_1x1 (model_partseg.py:15-92, use_cpu=True) on
                     (2,3,128) k=10, and Net (emb=64, 1 block, dropout 0) fwd +
                     bwd with its initial state_dict.
  hashes.json        SHA-256 of the canonical int32 kNN of the full-size bench
                     inputs (cfg2/cfg3/cfg5 first layer) + state_dict key lists.
"""
import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
import importlib.util  # noqa: E402

# repo-owned input generator, loaded by path so that `models` below is the reference's
_spec = importlib.util.spec_from_file_location("dgx_synth", os.path.join(REPO, "dgcnn.pytorch_amd", "dgx", "synth.py"))
synth = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(synth)

REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
from models.dgcnn import knn as ref_knn, get_graph_feature as ref_ggf, DGCNN as RefDGCNN  # noqa: E402
from models.layers import PositionEmbedding as RefPosEmb  # noqa: E402
import models.model_partseg as ref_partseg  # noqa: E402

torch.set_num_threads(8)


def ref_pd(x):
    inner = -2 * torch.matmul(x.transpose(2, 1).contiguous(), x)
    xx = torch.sum(x ** 2, dim=1, keepdim=True)
    return -xx - inner - xx.transpose(2, 1).contiguous()


def canonical(idx, pd):
    vals = torch.gather(pd, 2, idx)
    out_i, out_v = [], []
    idx_np, v_np = idx.numpy(), vals.numpy()
    order = np.lexsort((idx_np, -v_np), axis=-1)
    return np.take_along_axis(idx_np, order, 2), np.take_along_axis(v_np, order, 2)


def knn_cases():
    out = {}
    cases = [("c3", 3, 2, 256, 20), ("c9", 9, 2, 256, 20), ("c64", 64, 2, 256, 20), ("c128", 128, 2, 256, 20),
             ("c3k40", 3, 1, 512, 40), ("c64k32", 64, 1, 300, 32), ("c3n1000", 3, 2, 1000, 20)]
    for name, C, B, N, k in cases:
        for layout in ("bcn", "perm"):
            seed = 100 + C + N + k
            if C == 3:
                pts = synth.cube_clouds(B, N, seed)
            elif C == 9:
                pts = synth.s3dis_blocks(B, N, seed)
            else:
                pts = synth.relu_normal(seed, (B, N, C))
            t = torch.from_numpy(pts)
            x = t.permute(0, 2, 1) if layout == "perm" else t.permute(0, 2, 1).contiguous()
            idx = ref_knn(x, k)
            ci, cv = canonical(idx, ref_pd(x))
            key = f"{name}_{layout}"
            out[key + "_x"] = pts
            out[key + "_idx"] = ci.astype(np.int32)
            out[key + "_val"] = cv
    # ties: duplicated points
    pts = synth.tie_clouds(2, 256, seed=1, frac=0.05)
    x = torch.from_numpy(pts).permute(0, 2, 1)
    idx = ref_knn(x, 20)
    ci, cv = canonical(idx, ref_pd(x))
    out["ties_perm_x"], out["ties_perm_idx"], out["ties_perm_val"] = pts, ci.astype(np.int32), cv
    np.savez_compressed(os.path.join(HERE, "knn_cases.npz"), **out)


def graph_feature_cases():
    out = {}
    pts = synth.cube_clouds(2, 64, 21)
    x = torch.from_numpy(pts).permute(0, 2, 1).contiguous()
    feat = torch.from_numpy(synth.relu_normal(22, (2, 8, 64)))
    for name, inp in (("xyz", x), ("feat", feat)):
        out[name + "_x"] = inp.numpy()
        out[name + "_cat"] = ref_ggf(inp, k=8).numpy()
        out[name + "_disp"] = ref_ggf(inp, k=8, disp_only=True).numpy()
        out[name + "_knn"] = ref_ggf(inp, k=8, knn_only=True).numpy()
        ci, _ = canonical(ref_knn(inp, 8), ref_pd(inp))
        out[name + "_idx"] = ci.astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "graph_feature.npz"), **out)


def edgeconv_block_case():
    torch.manual_seed(3)
    B, C, N, k, Co = 2, 8, 128, 16, 32
    x = torch.from_numpy(synth.relu_normal(31, (B, C, N))).requires_grad_(True)
    block = torch.nn.Sequential(torch.nn.Conv2d(2 * C, Co, 1, bias=False), torch.nn.BatchNorm2d(Co),
                                torch.nn.LeakyReLU(0.2, inplace=True))
    with torch.no_grad():
        block[1].weight.copy_(torch.randn(Co))          # includes negative gammas
        block[1].bias.copy_(torch.randn(Co) * 0.1)
    w0 = block[0].weight.detach().clone()
    g0, b0 = block[1].weight.detach().clone(), block[1].bias.detach().clone()
    block.train()
    y = block(ref_ggf(x, k=k)).max(dim=-1, keepdim=False)[0]
    gy = torch.from_numpy(synth.uniform(32, tuple(y.shape)) - 0.5)
    y.backward(gy)
    ci, _ = canonical(ref_knn(x.detach(), k), ref_pd(x.detach()))
    np.savez_compressed(os.path.join(HERE, "edgeconv_block.npz"), x=x.detach().numpy(), idx=ci.astype(np.int32),
                        weight=w0.numpy(), gamma=g0.numpy(), beta=b0.numpy(), k=k, out=y.detach().numpy(),
                        gout=gy.numpy(), dx=x.grad.numpy(), dweight=block[0].weight.grad.numpy(),
                        dgamma=block[1].weight.grad.numpy(), dbeta=block[1].bias.grad.numpy(),
                        running_mean=block[1].running_mean.numpy(), running_var=block[1].running_var.numpy())


def dgcnn_case():
    torch.manual_seed(4)
    args = types.SimpleNamespace(emb_dim=64, k=10)
    model = RefDGCNN(args)
    state0 = {k_: v.detach().clone().numpy() for k_, v in model.state_dict().items()}
    x = torch.from_numpy(synth.cube_clouds(2, 128, 41)).permute(0, 2, 1)
    model.train()
    y = model(x)
    gy = torch.from_numpy(synth.uniform(42, tuple(y.shape)) - 0.5)
    y.backward(gy)
    grads = {"grad." + n: p.grad.numpy() for n, p in model.named_parameters()}
    after = {"after." + k_: v.numpy() for k_, v in model.state_dict().items() if "running" in k_}
    init = {"init." + k_: v for k_, v in state0.items()}
    np.savez_compressed(os.path.join(HERE, "dgcnn_small.npz"), x=x.contiguous().numpy(), out=y.detach().numpy(),
                        gout=gy.numpy(), **init, **grads, **after)


def posemb_case():
    """Weights are re-created from the seed by the test (same parameter
    construction order); the init state's SHA-256 pins that. Gradients of the
    two large dense weights are stored as projections to keep the fixture small."""
    torch.manual_seed(5)
    args = types.SimpleNamespace(k=10)
    model = RefPosEmb(args)
    with torch.no_grad():  # non-trivial transform so the bmm path is exercised
        model.transform.weight.normal_(0, 0.05)
    init_sha = hashlib.sha256(b"".join(v.detach().numpy().tobytes() for v in model.state_dict().values())).hexdigest()
    x = torch.from_numpy(synth.cube_clouds(4, 128, 51)).permute(0, 2, 1).contiguous()
    model.train()
    y = model(x)
    gy = torch.from_numpy(synth.uniform(52, tuple(y.shape)) - 0.5)
    y.backward(gy)
    big = ("conv3.0.weight", "linear.0.weight")
    grads, proj = {}, {}
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        if n in big:
            r = synth.uniform(53, tuple(p.shape)) - 0.5
            proj["gradproj." + n] = np.array([(p.grad.numpy().astype(np.float64) * r).sum(),
                                              np.linalg.norm(p.grad.numpy().astype(np.float64))])
        else:
            grads["grad." + n] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "posemb_small.npz"), x=x.numpy(), out=y.detach().numpy(),
                        gout=gy.numpy(), init_sha256=np.array(init_sha), **grads, **proj)


PARTSEG_BIG = ("pos_mlp.0.conv3.0.weight", "pos_mlp.0.linear.0.weight")


def partseg_big_init(i, shape):
    """Deterministic init of the large PositionEmbedding weights (tests redo this)."""
    return ((synth.uniform(63 + i, shape) - 0.5) * (2.0 / np.sqrt(shape[1]))).astype(np.float32)


def partseg_case():
    """HOG on its own, then a small Net. The reference's Net.forward calls
    compute_hog_1x1 with use_cpu=False (.cuda()); for this CPU-only run the
    module attribute is rebound in memory to the use_cpu=True variant."""
    x = torch.from_numpy(synth.cube_clouds(2, 128, 61)).permute(0, 2, 1).contiguous()
    hog = ref_partseg.compute_hog_1x1(x, 10, use_cpu=True)
    orig = ref_partseg.compute_hog_1x1
    ref_partseg.compute_hog_1x1 = lambda xx, k: orig(xx, k, use_cpu=True)
    try:
        torch.manual_seed(6)
        args = types.SimpleNamespace(emb_dim=64, k=10, n_heads=4, n_blocks=1, ff_dims=128, dropout=0.0,
                                     nclasses=50)
        model = ref_partseg.Net(args).train()
        with torch.no_grad():  # the two large weights come from the repo generator (not stored)
            for i, n in enumerate(PARTSEG_BIG):
                w = model.get_parameter(n)
                w.copy_(torch.from_numpy(partseg_big_init(i, tuple(w.shape))))
        state0 = {"init." + k_: v.detach().clone().numpy() for k_, v in model.state_dict().items()
                  if k_ not in PARTSEG_BIG and k_.replace("bn3", "conv3.1") not in PARTSEG_BIG}
        lbl = torch.zeros(2, 16)
        lbl[0, 3] = 1
        lbl[1, 11] = 1
        y = model(x, lbl)
        gy = torch.from_numpy(synth.uniform(62, tuple(y.shape)) - 0.5)
        y.backward(gy)
        grads = {"grad." + n: p.grad.numpy() for n, p in model.named_parameters()
                 if p.grad is not None and n not in PARTSEG_BIG}
        for i, n in enumerate(PARTSEG_BIG):
            gr = model.get_parameter(n).grad.numpy().astype(np.float64)
            r = synth.uniform(70 + i, gr.shape) - 0.5
            grads["gradproj." + n] = np.array([(gr * r).sum(), np.linalg.norm(gr)])
    finally:
        ref_partseg.compute_hog_1x1 = orig
    np.savez_compressed(os.path.join(HERE, "partseg_small.npz"), x=x.numpy(), hog=hog.numpy(), lbl=lbl.numpy(),
                        out=y.detach().numpy(), gout=gy.numpy(), **state0, **grads)


def hashes():
    res = {}
    for name, B, N, k, gen in (("cfg2_layer1", 32, 1024, 20, lambda: synth.cube_clouds(32, 1024, 0)),
                               ("cfg3_layer1", 32, 2048, 40, lambda: synth.cube_clouds(32, 2048, 0)),
                               ("cfg5_layer1", 24, 4096, 20, lambda: synth.s3dis_blocks(24, 4096, 2)),
                               ("ties_layer1", 32, 1024, 20, lambda: synth.tie_clouds(32, 1024, 1))):
        pts = gen()
        x = torch.from_numpy(pts).permute(0, 2, 1)
        idx = ref_knn(x, k)
        ci, cv = canonical(idx, ref_pd(x))
        # with exact ties at the k-th value the reference's index SET is arbitrary:
        # only the selected values are a valid comparator there (val_sha256)
        res[name] = {"B": B, "N": N, "k": k,
                     "input_sha256": hashlib.sha256(pts.tobytes()).hexdigest(),
                     "idx_sha256": hashlib.sha256(ci.astype(np.int32).tobytes()).hexdigest(),
                     "val_sha256": hashlib.sha256(cv.astype(np.float32).tobytes()).hexdigest(),
                     "boundary_ties": bool((cv[..., -1] == cv[..., -2]).any())}
        print(name, res[name]["idx_sha256"][:16])
    res["state_dict_keys"] = {
        "DGCNN": list(RefDGCNN(types.SimpleNamespace(emb_dim=1024, k=20)).state_dict().keys()),
        "PositionEmbedding": list(RefPosEmb(types.SimpleNamespace(k=20)).state_dict().keys()),
    }
    with open(os.path.join(HERE, "hashes.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1:] == ["partseg"]:
        partseg_case()
        sys.exit(0)
    knn_cases()
    graph_feature_cases()
    edgeconv_block_case()
    dgcnn_case()
    posemb_case()
    partseg_case()
    hashes()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
