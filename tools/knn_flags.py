"""Diagnostics: fraction of kNN rows the selection kernel flags for the exact
fix-up pass (run with DGX_KNN_NOFIX=1 so the markers stay visible)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import synth  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402

dev = torch.device("cuda:0")
x3 = torch.from_numpy(synth.cube_clouds(32, 1024, 0)).to(dev).permute(0, 2, 1)
f64 = torch.from_numpy(synth.relu_normal(3, (32, 64, 1024))).to(dev)
for name, x in (("C3", x3), ("C64", f64)):
    idx, vals = knn_raw(x, 20, out_dtype=torch.int32, return_values=True)
    fl = idx[:, :, 0] < 0
    print(name, "flagged rows", int(fl.sum()), "of", fl.numel())
    if fl.any():
        r = fl.nonzero()[0]
        print(" first flagged", r.tolist(), "row idx", idx[r[0], r[1]].tolist()[:6], "vals", vals[r[0], r[1]].tolist()[:4])
        import struct
        print(" T0 bits as float", struct.unpack("f", struct.pack("i", int(idx[r[0], r[1], 1])))[0])
