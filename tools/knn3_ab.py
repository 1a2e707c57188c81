"""A/B of the 3-channel kNN selection: knn3_kernel (VALU, lane = query) vs the
MFMA selection kernel, interleaved, on the xyz shapes of cfg2 / cfg4 layer 1
and the HOG / PositionEmbedding kNN; outputs of both must be identical.
    python tools/knn3_ab.py [reps]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import _native as nat  # noqa: E402
from dgx import synth  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")
L = nat.lib()
cases = [("C3 B32 N1024 k20", 32, 1024, 20), ("C3 B32 N2048 k40", 32, 2048, 40), ("C3 B32 N2048 k20", 32, 2048, 20),
         ("C3 B8 N4096 k20", 8, 4096, 20), ("C3 B4 N777 k16", 4, 777, 16)]
for name, B, N, k in cases:
    x = torch.from_numpy(synth.cube_clouds(B, N, 7)).to(dev).permute(0, 2, 1)
    res, outs = {0: [], 1: []}, {}
    for v in (0, 1):
        L.dgx_knn_set_variant(v)
        outs[v] = knn_raw(x, k, out_dtype=torch.int32, return_values=True)
    for rnd in range(5):
        for v in (0, 1):
            L.dgx_knn_set_variant(v)
            for _ in range(3):
                knn_raw(x, k, out_dtype=torch.int32)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                knn_raw(x, k, out_dtype=torch.int32)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / reps * 1e3)
    L.dgx_knn_set_variant(1)
    same = torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    med = {v: sorted(t)[len(t) // 2] for v, t in res.items()}
    print(f"{name}: mfma {med[0]:.1f} us/call, knn3 {med[1]:.1f} us/call (incl. image pass); identical idx: {same}",
          flush=True)
