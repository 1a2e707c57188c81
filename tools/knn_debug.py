"""Debug driver (not product): repeated engine kNN on the adversarial 1-/2-
channel clouds; reports rows that differ between calls or from the oracle."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd"), os.path.join(REPO, "tests")]
import oracle  # noqa: E402
from dgx import synth  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402

dev = torch.device("cuda:0")
for C in (1, 2, 3):
    B, N, k = 3, 777, 16
    pts = synth.cube_clouds(B, N, 40 + C)[..., :C].copy()
    f = torch.from_numpy(pts).permute(0, 2, 1).contiguous()
    ref_idx, ref_vals = oracle.knn(f, k, return_values=True)
    ref_idx, ref_vals = np.asarray(ref_idx), np.asarray(ref_vals)
    x = f.to(dev)
    for rep in range(4):
        idx, vals = knn_raw(x, k, return_values=True)
        i32 = knn_raw(x, k, out_dtype=torch.int32)
        idx, vals, i32 = idx.cpu().numpy(), vals.cpu().numpy(), i32.cpu().numpy()
        bad = np.argwhere((idx != ref_idx).any(-1))
        bad32 = np.argwhere((i32 != ref_idx).any(-1))
        badv = np.argwhere((vals != ref_vals).any(-1))
        print(f"C{C} rep{rep}: rows != oracle: int64 {len(bad)} int32 {len(bad32)} vals {len(badv)}", flush=True)
        for (b, q) in list(bad[:2]) + list(bad32[:1]):
            print(f"   b{b} q{q} i64 {idx[b, q]}\n          i32 {i32[b, q]}\n          ref {ref_idx[b, q]}"
                  f"\n     vals {vals[b, q]}\n     refv {ref_vals[b, q]}", flush=True)
