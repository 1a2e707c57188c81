"""Debug helper: GPU kNN vs oracle on the full-size bench inputs, row diagnostics."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import oracle  # noqa: E402
from dgx import synth  # noqa: E402
from models.dgcnn import knn  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402

cases = {"cfg2": (synth.cube_clouds(32, 1024, 0), 20), "ties": (synth.tie_clouds(32, 1024, 1), 20),
         "cfg3": (synth.cube_clouds(32, 2048, 0), 40)}
for name, (pts, k) in cases.items():
    x = torch.from_numpy(pts).permute(0, 2, 1)
    gi, gv = knn_raw(x.cuda(), k, return_values=True)
    gi, gv = gi.cpu().numpy(), gv.cpu().numpy()
    oi = oracle.knn(x, k)
    bad = np.argwhere((gi != oi).any(-1))
    print(name, "bad rows", len(bad))
    for b, i in bad[:6]:
        pd = oracle.pairwise(x[b:b + 1])[0, i]
        print(" row", b, i)
        print("  gpu", gi[b, i].tolist())
        print("  ora", oi[b, i].tolist())
        print("  gpu vals", [float(pd[j]) for j in gi[b, i]])
        print("  gpu own vals", gv[b, i].tolist())
        print("  ora vals", [float(pd[j]) for j in oi[b, i]])
