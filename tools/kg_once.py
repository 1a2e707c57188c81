"""A few grid-kNN calls at cfg2 block-1 geometry (for PMC / kernel-trace passes)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import synth  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402

dev = torch.device("cuda:0")
B, N, k = (32, 2048, 40) if len(sys.argv) > 1 and sys.argv[1] == "k40" else (32, 1024, 20)
x = torch.from_numpy(synth.cube_clouds(B, N, 0)).to(dev).permute(0, 2, 1)
for _ in range(5):
    knn_raw(x, k, out_dtype=torch.int32)
torch.cuda.synchronize()
