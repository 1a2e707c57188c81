"""PositionEmbedding edge-MLP leg of bench.py on its own (for rocprofv3 runs):
python tools/posemb_bench.py [--fp32] [--no-eager]."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from dgx import precision  # noqa: E402

if __name__ == "__main__":
    precision.set("fp32" if "--fp32" in sys.argv else "bf16")
    dev = torch.device("cuda:0")
    if "--no-eager" in sys.argv:
        from dgx.edgemlp import edge_mlp2  # noqa: F401
        bench_out = {"engine_only": True}
        import torch.nn as nn
        x = (torch.rand(32, 3, 2048, device=dev) * 2 - 1).requires_grad_(True)
        c1 = nn.Sequential(nn.Conv2d(6, 64, 1, bias=False), nn.BatchNorm2d(64), nn.LeakyReLU(0.2)).to(dev)
        c2 = nn.Sequential(nn.Conv2d(64, 128, 1, bias=False), nn.BatchNorm2d(128), nn.LeakyReLU(0.2)).to(dev)
        g = torch.randn(32, 128, 2048, device=dev)
        for _ in range(6):
            edge_mlp2(x, 40, c1, c2, True).backward(g)
        torch.cuda.synchronize()
    else:
        bench_out = bench.posemb_edge_leg(dev)
    print(json.dumps({"precision": precision.get(), **bench_out}), flush=True)
