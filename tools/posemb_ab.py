"""A/B of the PositionEmbedding edge stage (bench.py's posemb leg, engine only:
B 32, N 2048, k 40, bf16, fwd+bwd) with the fused and the unfused edge-MLP
backward (dgx.edgemlp.FUSED_BWD), interleaved: python tools/posemb_ab.py [rounds]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import bench  # noqa: E402
import dgx.edgemlp as EM  # noqa: E402
from dgx import precision  # noqa: E402

dev = torch.device("cuda:0")
precision.set("bf16")
torch.manual_seed(1)
B, N, k = 32, 2048, 40
c1 = nn.Sequential(nn.Conv2d(6, 64, 1, bias=False), nn.BatchNorm2d(64), nn.LeakyReLU(0.2)).to(dev)
c2 = nn.Sequential(nn.Conv2d(64, 128, 1, bias=False), nn.BatchNorm2d(128), nn.LeakyReLU(0.2)).to(dev)
x = (torch.rand(B, 3, N, device=dev) * 2 - 1).requires_grad_(True)
g = torch.randn(B, 128, N, device=dev)


def engine():
    EM.edge_mlp2(x, k, c1, c2).backward(g)


res = {True: [], False: []}
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    for flag in (False, True):
        EM.FUSED_BWD = flag
        res[flag].append(bench._ms(engine, 5, warm=1))
for flag, ms in res.items():
    ms = sorted(ms)
    print(f"FUSED_BWD={flag}: median {ms[len(ms) // 2]:.3f} ms  all {' '.join(f'{m:.3f}' for m in res[flag])}",
          flush=True)
