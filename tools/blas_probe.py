"""Times torch's library GEMM (hipBLASLt) on conv5's three shapes at cfg2
(M = B*N = 32768 rows, emb 1024, K = 512) as a yardstick for the engine's
gemm256 / gemm_lds kernels (bf16 operands, fp32 accumulate)."""
import torch

def t(fn, it=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1000

dev = "cuda"
M, E, K = 32768, 1024, 512
X = torch.randn(M, K, device=dev).bfloat16()
W = torch.randn(E, K, device=dev).bfloat16()
dZ = torch.randn(M, E, device=dev).bfloat16()
fl = 2 * M * E * K / 1e12
for name, fn in [("fwd Z = X W^T (bf16 out)", lambda: X @ W.t()),
                 ("fwd Z fp32 out", lambda: torch.matmul(X, W.t()).float()),
                 ("dX = dZ W", lambda: dZ @ W),
                 ("dW = dZ^T X", lambda: dZ.t() @ X)]:
    us = t(fn)
    print(f"{name:28s} {us:7.1f} us  {fl / (us * 1e-6):7.1f} TF/s")
