"""One PositionEmbedding edge stage fwd+bwd at cfg4 geometry (B 32, N 2048, k 40, bf16), a few
repetitions, for rocprofv3 runs: python tools/posemb_once.py [fused 0|1] [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import dgx.edgemlp as EM  # noqa: E402
from dgx import precision  # noqa: E402

EM.FUSED_BWD = bool(int(sys.argv[1])) if len(sys.argv) > 1 else True
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
precision.set("bf16")
torch.manual_seed(1)
c1 = nn.Sequential(nn.Conv2d(6, 64, 1, bias=False), nn.BatchNorm2d(64), nn.LeakyReLU(0.2)).to(dev)
c2 = nn.Sequential(nn.Conv2d(64, 128, 1, bias=False), nn.BatchNorm2d(128), nn.LeakyReLU(0.2)).to(dev)
x = (torch.rand(32, 3, 2048, device=dev) * 2 - 1).requires_grad_(True)
g = torch.randn(32, 128, 2048, device=dev)
for _ in range(reps):
    EM.edge_mlp2(x, 40, c1, c2).backward(g)
torch.cuda.synchronize()
print("done")
