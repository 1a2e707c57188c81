"""Dump the fused edge-MLP forward (bf16 mode) outputs for a variant library,
to compare kernel variants bit for bit across DGX_LIB builds:
  DGX_LIB=... python tools/emf_dump.py out.pt"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import dgx.edgemlp as EM  # noqa: E402
from dgx import precision  # noqa: E402

dev = torch.device("cuda:0")
precision.set("bf16")
out = {}
for B, N, k in [(4, 2048, 40), (2, 300, 33), (3, 130, 9), (2, 1024, 20), (1, 77, 64)]:
    torch.manual_seed(B * 1000 + N + k)
    c1 = nn.Sequential(nn.Conv2d(6, 64, 1, bias=False), nn.BatchNorm2d(64), nn.LeakyReLU(0.2)).to(dev)
    c2 = nn.Sequential(nn.Conv2d(64, 128, 1, bias=False), nn.BatchNorm2d(128), nn.LeakyReLU(0.2)).to(dev)
    with torch.no_grad():
        c2[1].weight.copy_(torch.randn(128))  # negative gammas: the min branch too
    x = (torch.rand(B, 3, N, device=dev) * 2 - 1).requires_grad_(True)
    y = EM.edge_mlp2(x, k, c1, c2, True)
    y.backward(torch.randn_like(y))
    out[f"{B},{N},{k}"] = {"y": y.detach().cpu(), "rm": c2[1].running_mean.cpu(), "rv": c2[1].running_var.cpu(),
                           "gx": x.grad.cpu(), "gw2": c2[0].weight.grad.cpu()}
torch.save(out, sys.argv[1])
print("saved", sys.argv[1])
