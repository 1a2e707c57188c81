"""Per-row diagnostics of knn_bf_kernel (diagnostics build, KNN_BF_DIAG):
flag reasons (1 = exact list full, 2 = FIFO overflow, 4 = non-finite bound),
the bound eps, the final admission bound, the merged k-th value, FIFO fill."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import synth  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402

dev = torch.device("cuda:0")
for name, C, seed in (("C64", 64, 3), ("C128", 128, 4)):
    f = torch.from_numpy(synth.relu_normal(seed, (4, C, 1024))).to(dev)
    _, vals = knn_raw(f, 20, return_values=True)
    v = vals.view(-1, 20)[:, :5].cpu().numpy()
    why = v[:, 0].astype(int)
    print(name, "rows", len(v), "flag=1:", (why & 1).astype(bool).sum(), "flag=2:", (why & 2).astype(bool).sum(),
          "flag=4:", (why & 4).astype(bool).sum())
    print("  eps mean %.4f  bound-kth mean %.4f  fifo max mean %.2f max %d" % (
        v[:, 1].mean(), (v[:, 2] - v[:, 3]).mean(), v[:, 4].mean(), v[:, 4].max()))
    print("  sample rows:", np.round(v[:4], 4).tolist())
