"""Count the rows knn_kernel flags for the exact fix-up (rank-0 id = -1 before
knn_fix_kernel) on the layer inputs the bench's training loop produces.

  python tools/knn_flag_probe.py <probe build of libdgx without the fix-up launch>
"""
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import torch  # noqa: E402

from dgx import ops, precision, synth  # noqa: E402


def probe(path, steps=45):
    """Run the bench's training loop (bf16, lr 0.1, its upstream gradient) and
    re-run every kNN call through the probe library ``path`` (a build without
    the fix-up launch) to count the rows the selection flagged."""
    import ctypes
    import bench
    from dgx import _native as nat
    from dgx import edgeconv
    from models.dgcnn import DGCNN
    dev = torch.device("cuda:0")
    probe_lib = ctypes.CDLL(path)
    for name, argtypes in nat._SIGS.items():
        fn = getattr(probe_lib, name)
        fn.argtypes = argtypes
        fn.restype = nat._RESTYPES.get(name, ctypes.c_int)
    precision.set("bf16")
    torch.manual_seed(0)
    m = DGCNN(types.SimpleNamespace(emb_dim=1024, k=20, in_dims=3)).to(dev).train()
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.from_numpy(synth.cube_clouds(32, 1024, 0)).to(dev).permute(0, 2, 1)
    gy = bench.upstream_grad((32, 1024, 1024), dev)
    real = edgeconv.knn_raw
    flags = []

    def spy(xin, k, **kw):
        out = real(xin, k, **kw)
        keep = nat.lib()
        nat._lib = probe_lib
        try:
            idx = real(xin, k, **kw)
        finally:
            nat._lib = keep
        flags.append(int((idx.view(-1, k)[:, 0] == -1).sum()))
        return out

    edgeconv.knn_raw = spy
    for s in range(steps):
        flags.clear()
        opt.zero_grad(set_to_none=True)
        m(x).backward(gy)
        opt.step()
        torch.cuda.synchronize()
        print("step", s, "flagged rows per block", flags, flush=True)


if __name__ == "__main__":
    probe(sys.argv[1])
