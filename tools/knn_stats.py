"""Selection diagnostics of the kNN kernel (insertion rounds, flushes and
flagged rows per wave), with and without spatial seeds, from a diagnostics build of knn.hip:
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DDGX_KNN_STATS -shared \
        dgcnn.pytorch_amd/csrc/*.hip -o /tmp/libdgx_stats.so
    DGX_LIB=/tmp/libdgx_stats.so python tools/knn_stats.py"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import _native as nat  # noqa: E402
from dgx import synth  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402

dev = torch.device("cuda:0")
L = nat.lib()
L.dgx_knn_stats_buffer.argtypes = [ctypes.c_void_p]
L.dgx_knn_stats_buffer.restype = None
from dgx import ops  # noqa: E402
for sort, name, B, N, k, C in [(o,) + c for o in (0, 1) for c in (("C3 N1024 k20", 32, 1024, 20, 3), ("C3 N2048 k40", 32, 2048, 40, 3))]:
    ops.SPATIAL_SEEDS = bool(sort)
    x = torch.from_numpy(synth.cube_clouds(B, N, 0)).to(dev).permute(0, 2, 1)
    nqb = (N + 31) // 32
    blocks = 8 * ((B + 7) // 8) * nqb
    st = torch.zeros(blocks * 4 * 4, dtype=torch.int32, device=dev)
    L.dgx_knn_stats_buffer(st.data_ptr())
    knn_raw(x, k, out_dtype=torch.int32)
    torch.cuda.synchronize()
    v = st.view(-1, 4).cpu().long()
    live = v[:, 3] == 1
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(10):
        knn_raw(x, k, out_dtype=torch.int32)
    ev1.record()
    torch.cuda.synchronize()
    print(f"spatial_seeds={sort} {name}: {ev0.elapsed_time(ev1) / 10 * 1e3:.1f} us/call; waves {int(live.sum())}, insertion rounds/wave {v[live, 0].float().mean():.1f}, "
          f"flushes/wave {v[live, 1].float().mean():.1f}, flagged rows {int(v[:, 2].sum())} of {B * N}")
