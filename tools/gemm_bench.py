"""Time the engine's bf16 GEMMs at the conv5 shapes of the headline config
(M = 32*1024 points, K = 512 concat channels, N = emb 1024): forward with the
BN-statistics + bf16 epilogue, input gradient, weight gradient. HIP-event
timing over `reps` launches; prints TF/s and the fraction of the 2.5 PF bf16
dense peak. Diagnostic (tools/), not part of the product."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import gemm as G  # noqa: E402

M, K, N = 32768, 512, 1024
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")
torch.manual_seed(0)
x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
wt = w.t().contiguous()
dz = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16)
dw = torch.empty(N, K, device=dev)


def t(fn, flops):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    tf = flops / us / 1e6
    return us, tf


zo = torch.empty(M, N, device=dev)
for name, fn in (("conv5 fwd Z=X W^T +stats bf16", lambda: G.lds_xwt(x, w, stats=True, out_bf16=True)),
                 ("conv5 fwd Z=X W^T fp32 store", lambda: G.lds_xwt(x, w, out=zo)),
                 ("conv5 fwd Z=X W^T fp32 +stats", lambda: G.lds_xwt(x, w, stats=True)),
                 ("conv5 dX = dZ W", lambda: G.lds_xwt(dz, wt)),
                 ("conv5 dW = dZ^T X", lambda: G.lds_atb(dz, x, dw))):
    us, tf = t(fn, 2.0 * M * N * K)
    print(f"{name:32s} {us:8.1f} us  {tf:7.1f} TF/s  {tf / 2500:.3f} of bf16 dense peak")
