"""Stage timing of the grid kNN (diagnostics builds tools/diag/libdgx_kg<S>.so,
-DDGX_KG_STAGE=S early exits): DGX_LIB=... python tools/kg_stage.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import _native as nat  # noqa: E402
from dgx import synth  # noqa: E402

dev = torch.device("cuda:0")
for B, N, k in ((32, 1024, 20), (32, 2048, 40)):
    x = torch.from_numpy(synth.cube_clouds(B, N, 0)).to(dev).permute(0, 2, 1)
    idx = torch.empty((B, N, k), dtype=torch.int32, device=dev)
    vals = torch.zeros((B, N, k), dtype=torch.float32, device=dev)
    L = nat.lib()

    def call():
        nat.check(L.dgx_knn_grid_f32(nat.f32(x), *x.stride(), B, 3, N, k, None, nat.i32(idx), nat.f32(vals),
                                     nat.stream_of(x)), "grid")
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        call()
    e1.record()
    torch.cuda.synchronize()
    nblk = 8 * ((B + 7) // 8) * ((N + 63) // 64)
    flagged = float(vals.view(-1)[:nblk * 4].sum()) if "kg4" in os.environ.get("DGX_LIB", "") else -1
    print(f"{os.path.basename(os.environ.get('DGX_LIB', 'libdgx.so'))} B={B} N={N} k={k}: "
          f"{e0.elapsed_time(e1) / 20 * 1e3:.1f} us; flagged queries {flagged}", flush=True)
