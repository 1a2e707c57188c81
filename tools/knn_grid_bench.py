"""Time the coordinate-cloud kNN: the cell-grid kernel (one launch) against the
dense path (image pass + MFMA selection) at the bench geometries, HIP events
on the launch stream. python tools/knn_grid_bench.py [reps]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd"), os.path.join(REPO, "tests")]
from dgx import synth  # noqa: E402
from test_knn_grid_gpu import _clouds, _dense, _grid  # noqa: E402


def grid_call(x, k, idx):
    from dgx import _native as nat
    B, C, N = x.shape
    nat.check(nat.lib().dgx_knn_grid_f32(nat.f32(x), *x.stride(), B, C, N, k, None, nat.i32(idx), None,
                                         nat.stream_of(x)), "grid")


def timed(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    for name, B, N, k, kind in (("cfg2 block1", 32, 1024, 20, "cube"), ("cfg3/cfg4 k40", 32, 2048, 40, "cube"),
                                ("cfg4 surface k40", 32, 2048, 40, "surface"), ("N4096 k20", 24, 4096, 20, "cube"),
                                ("B4 shard", 4, 1024, 20, "cube")):
        x = torch.from_numpy(_clouds(kind, B, N, 0) if kind != "cube" else synth.cube_clouds(B, N, 0)).to(dev)
        x = x.permute(0, 2, 1)
        i32 = torch.empty((B, N, k), dtype=torch.int32, device=dev)
        tg = timed(lambda: grid_call(x, k, i32), reps)
        td = timed(lambda: _dense(x, k), reps)
        same = torch.equal(_grid(x, k)[0], _dense(x, k)[0])
        flops = 2.0 * B * N * N * 3
        print(f"{name:18s} B={B} N={N} k={k}: grid {tg:7.1f} us ({flops / tg / 1e6:6.1f} TF/s dense-equiv), "
              f"dense {td:7.1f} us, identical={same}", flush=True)


if __name__ == "__main__":
    main()
