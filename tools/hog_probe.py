"""f1 probe on the GPU box: agreement of dgx_hog_1x1_f32 with the oracle's
restatement of the reference (exact-point fraction, max abs diff) and timing
of the device HOG vs the reference's host round trip (D2H + numpy SVD + H2D +
torch votes), at the partseg configuration (B=32, N=2048, k=20).

  python tools/hog_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "dgcnn.pytorch_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from dgx.hog import hog_1x1  # noqa: E402
from models.dgcnn import knn  # noqa: E402
from oracle.hog import hog_1x1 as ref_hog  # noqa: E402


def main():
    dev = torch.device("cuda")
    for B, N, k in ((32, 2048, 20), (8, 2048, 40), (16, 1024, 10)):
        x = (torch.rand((B, 3, N), generator=torch.Generator().manual_seed(B + k)) * 2 - 1)
        xd = x.to(dev)
        idx = knn(xd, k)
        got = hog_1x1(xd, idx)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            got = hog_1x1(xd, idx)
        torch.cuda.synchronize()
        dt_dev = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        ref = ref_hog(x, idx.cpu())
        dt_ref = time.perf_counter() - t0
        g, r = got.cpu().numpy(), ref.numpy()
        exact = (g == r).all(-1).mean()
        print(f"B={B} N={N} k={k}: exact points {exact:.6f}, max|d| {np.abs(g - r).max():.3e}, "
              f"device {dt_dev * 1e3:.3f} ms, reference CPU path {dt_ref * 1e3:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
