"""Standalone kNN kernel driver for profiling (cfg2 layer shapes)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import synth  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
x3 = torch.from_numpy(synth.cube_clouds(32, 1024, 0)).to(dev).permute(0, 2, 1)
f64 = torch.from_numpy(synth.relu_normal(3, (32, 64, 1024))).to(dev)
f128 = torch.from_numpy(synth.relu_normal(4, (32, 128, 1024))).to(dev)
# point-major (B,N,C) memory, as the engine's concat buffer feeds layers 2-4
p64 = f64.permute(0, 2, 1).contiguous().permute(0, 2, 1)
p128 = f128.permute(0, 2, 1).contiguous().permute(0, 2, 1)
x3b = torch.from_numpy(synth.cube_clouds(32, 2048, 1)).to(dev).permute(0, 2, 1)
big = os.environ.get("KNN_BENCH_BIG") == "1"
cases = [("C3", x3, 20), ("C3 N2048 k40", x3b, 40), ("C64", f64, 20), ("C128", f128, 20),
         ("C64pm", p64, 20), ("C128pm", p128, 20)]
if big:  # cfg3 / cfg5 layer shapes (point-major, as the concat buffer feeds them)
    def pm(seed, shape):
        f = torch.from_numpy(synth.relu_normal(seed, shape)).to(dev)
        return f.permute(0, 2, 1).contiguous().permute(0, 2, 1)
    cases = [("C64 N2048 k40", pm(5, (32, 64, 2048)), 40), ("C128 N2048 k40", pm(6, (32, 128, 2048)), 40),
             ("C64 N4096", pm(7, (24, 64, 4096)), 20), ("C128 N4096", pm(8, (24, 128, 4096)), 20)]
for name, x, k in cases:
    for _ in range(3):
        knn_raw(x, k, out_dtype=torch.int32)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        knn_raw(x, k, out_dtype=torch.int32)
    ev1.record()
    torch.cuda.synchronize()
    print(name, "%.1f us/call (incl. sqnorm)" % (ev0.elapsed_time(ev1) / reps * 1e3))
