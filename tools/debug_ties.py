import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx.ops import knn_raw  # noqa
for N, k in ((64, 20), (256, 20), (1024, 20), (1024, 40), (100, 16)):
    x = torch.ones(1, 3, N, device="cuda") * 0.25
    idx, vals = knn_raw(x, k, return_values=True)
    idx = idx.cpu().numpy()[0]
    exp = np.arange(k)
    bad = np.argwhere((idx != exp).any(-1)).ravel()
    print(N, k, "rows wrong:", len(bad), "vals unique:", np.unique(vals.cpu().numpy()))
    for r in bad[:4]:
        print("  row", r, idx[r].tolist())
# two-level ties: points come in 4 distinct positions
N = 256
pos = torch.tensor([[0.0, 0, 0], [0.5, 0, 0], [0, 0.75, 0], [0, 0, 1.0]])
x = pos[torch.arange(N) % 4].t().unsqueeze(0).contiguous().cuda()
idx = knn_raw(x, 40).cpu().numpy()[0]
for r in (0, 1, 5):
    print("grp row", r, idx[r].tolist())
