"""Time the fused edge-MLP forward kernel with and without the h1 store (cfg4:
B 32, N 2048, k 40, conv 6 -> 64 -> 128): python tools/emlp_fwd_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from dgx import precision  # noqa: E402
from dgx.edgemlp import edge_mlp2  # noqa: E402

precision.set("bf16")
dev = torch.device("cuda:0")
x = (torch.rand(32, 3, 2048, device=dev) * 2 - 1)
c1 = nn.Sequential(nn.Conv2d(6, 64, 1, bias=False), nn.BatchNorm2d(64), nn.LeakyReLU(0.2)).to(dev)
c2 = nn.Sequential(nn.Conv2d(64, 128, 1, bias=False), nn.BatchNorm2d(128), nn.LeakyReLU(0.2)).to(dev)
for grad in (False, True):
    for _ in range(4):
        if grad:
            edge_mlp2(x.requires_grad_(True), 40, c1, c2, True)
        else:
            with torch.no_grad():
                edge_mlp2(x, 40, c1, c2, True)
torch.cuda.synchronize()
print("done")
