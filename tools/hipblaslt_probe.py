"""hipBLASLt (torch.mm) vs the engine's gemm256 at conv5's input-gradient shape:
dX (32768 x 512, fp32 out) = dZ (32768 x 1024 bf16) @ W (1024 x 512 bf16)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import torch  # noqa: E402

from dgx import gemm as G  # noqa: E402

dev = torch.device("cuda:0")


def t(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


M, K, N = 32768, 1024, 512
dZ = torch.randn(M, K, device=dev).to(torch.bfloat16)
W = torch.randn(K, N, device=dev).to(torch.bfloat16)       # dX = dZ W
wprep = G.prep_weight(torch.randn(K, N, device=dev), K, N, False)
Wt = wprep[1]                                                # (N, K) bf16: the engine's NT operand
fl = 2 * M * N * K
ref = torch.mm(dZ.float(), Wt.float().t())
for name, fn in (("hipBLASLt bf16 out", lambda: dZ @ Wt.t()),
                 ("hipBLASLt fp32 out", lambda: torch.mm(dZ, Wt.t(), out_dtype=torch.float32)),
                 ("engine gemm256 fp32 out", lambda: G.lds_xwt(dZ, Wt))):
    us = t(fn)
    err = float((fn().float() - ref).norm() / ref.norm())
    print(f"{name:26s} {us:7.1f} us  {fl / us / 1e6:7.1f} TFLOP/s  rel err {err:.1e}", flush=True)
