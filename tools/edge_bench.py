"""Standalone EdgeConv-chain driver (DGCNN blocks 1-4 fwd+bwd, cfg2) for profiling."""
import os
import sys
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import synth  # noqa: E402
from dgx.edgeconv import edgeconv_stack  # noqa: E402
from models.dgcnn import DGCNN  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = DGCNN(types.SimpleNamespace(emb_dim=1024, k=20)).to(dev).train()
x = torch.from_numpy(synth.cube_clouds(32, 1024, 0)).to(dev).permute(0, 2, 1)
for _ in range(reps):
    y = edgeconv_stack(x, 20, m.edge_blocks(), True)
    y.sum().backward()
torch.cuda.synchronize()
print("done", reps)
