"""Isolate the dPQ discrepancy: single blocks and 2-block stacks vs fp64 autograd."""
import os, sys
import numpy as np
import torch
import torch.nn.functional as Fn
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd"), os.path.join(REPO, "tests")]
from conftest import rel_err  # noqa
from oracle import reference as R  # noqa
from models.dgcnn import knn  # noqa
from dgx.edgeconv import edgeconv_stack  # noqa
dev = torch.device("cuda:0")


def mk(cin, co, gamma_mode, seed):
    torch.manual_seed(seed)
    blk = torch.nn.Sequential(torch.nn.Conv2d(2 * cin, co, 1, bias=False), torch.nn.BatchNorm2d(co),
                              torch.nn.LeakyReLU(0.2, inplace=True))
    if gamma_mode == "rand":
        with torch.no_grad():
            blk[1].weight.copy_(torch.randn(co)); blk[1].bias.copy_(0.1 * torch.randn(co))
    return blk


def run(widths, N, k, gamma_mode, B=2, seed=0):
    torch.manual_seed(seed)
    x = torch.randn(B, widths[0], N)
    blocks = [mk(a, b, gamma_mode, seed + i) for i, (a, b) in enumerate(zip(widths[:-1], widths[1:]))]
    gblocks = [torch.nn.Sequential(*[torch.nn.Conv2d(2 * a, b, 1, bias=False), torch.nn.BatchNorm2d(b),
                                     torch.nn.LeakyReLU(0.2, inplace=True)]) for a, b in zip(widths[:-1], widths[1:])]
    for gb, b in zip(gblocks, blocks):
        gb.load_state_dict(b.state_dict())
    gblocks = [b.to(dev) for b in gblocks]
    out = edgeconv_stack(x.to(dev), k, gblocks, True)
    gout = torch.randn(out.shape)
    out.backward(gout.to(dev))
    # fp64 reference with the GPU's neighbour sets
    feats = out.detach().cpu().view(B, N, -1).permute(0, 2, 1)
    h = x.double()
    ws = [p[0].weight.detach().double().requires_grad_(True) for p in blocks]
    gs = [p[1].weight.detach().double().requires_grad_(True) for p in blocks]
    bs = [p[1].bias.detach().double().requires_grad_(True) for p in blocks]
    hs, off = [], 0
    for li in range(len(blocks)):
        if li == 0:
            idx = knn(x.to(dev), k).cpu()
        else:
            prev = feats[:, off - widths[li]: off].contiguous()
            idx = knn(prev.to(dev), k).cpu()
        bn = {"weight": gs[li], "bias": bs[li], "running_mean": torch.zeros(widths[li + 1], dtype=torch.float64),
              "running_var": torch.ones(widths[li + 1], dtype=torch.float64)}
        h = R.edgeconv_block(h, k, ws[li], bn, True, idx=idx)
        hs.append(h)
        off += widths[li + 1]
    ref = torch.cat(hs, 1).permute(0, 2, 1).reshape(B * N, -1)
    ref.backward(gout.double())
    res = [f"fwd {rel_err(out.detach().cpu(), ref.detach()):.1e}"]
    for li, gb in enumerate(gblocks):
        res.append(f"L{li+1}: dW {rel_err(gb[0].weight.grad.cpu(), ws[li].grad):.1e} dg {rel_err(gb[1].weight.grad.cpu(), gs[li].grad):.1e} db {rel_err(gb[1].bias.grad.cpu(), bs[li].grad):.1e}")
    print(widths, N, k, gamma_mode, " | ".join(res))


for N in (128, 130):
    for gm in ("ones", "rand"):
        run([128, 256], N, 10, gm)
        run([64, 128, 256], N, 10, gm)
        run([3, 64], N, 10, gm)
run([3, 64, 64, 128, 256], 128, 10, "ones")
run([3, 64, 64, 128, 256], 1024, 20, "ones")
