"""Time the engine attention (dgx.attention) against torch's
scaled_dot_product_attention at Net's shape (BASELINE cfg4 per GPU: B 32,
N 2048, emb 512, 4 heads -> D 128, dropout 0.5).

  python tools/attn_bench.py [--batch 32] [--points 2048] [--emb 512] [--heads 4] [--dropout 0.5]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timed(fn, reps, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--points", type=int, default=2048)
    ap.add_argument("--emb", type=int, default=512)
    ap.add_argument("--heads", type=int, default=4)
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()
    from dgx.attention import attention
    dev = torch.device("cuda:0")
    B, N, E, H = a.batch, a.points, a.emb, a.heads
    D = E // H
    flops_fwd = 4.0 * B * H * N * N * D
    out = {"shape": {"B": B, "N": N, "E": E, "H": H, "D": D, "dropout": a.dropout}}
    for dt in (torch.float16, torch.bfloat16):
        g = torch.Generator(device=dev).manual_seed(0)
        qkv = torch.randn((B, N, 3 * E), device=dev, generator=g).to(dt)
        q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
        qg, kg, vg = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
        go = torch.randn((B, N, E), device=dev, generator=g).to(dt)
        r = {}
        r["engine_fwd_ms"] = timed(lambda: attention(q, k, v, H, a.dropout), a.reps)

        def eng_step():
            o = attention(qg, kg, vg, H, a.dropout)
            o.backward(go)
        r["engine_fwd_bwd_ms"] = timed(eng_step, a.reps)
        if not a.no_torch:
            def th(t):
                return t.reshape(B, N, H, D).transpose(1, 2)
            qt, kt, vt = (th(t) for t in (q, k, v))
            r["torch_sdpa_fwd_ms"] = timed(lambda: F.scaled_dot_product_attention(qt, kt, vt, dropout_p=a.dropout),
                                           a.reps)
            qh, kh, vh = (th(t).detach().clone().requires_grad_(True) for t in (q, k, v))
            goh = th(go)

            def th_step():
                o = F.scaled_dot_product_attention(qh, kh, vh, dropout_p=a.dropout)
                o.backward(goh)
            r["torch_sdpa_fwd_bwd_ms"] = timed(th_step, a.reps)
        r["engine_fwd_tflops"] = flops_fwd / (r["engine_fwd_ms"] * 1e-3) / 1e12
        # algorithmic: fwd 2 products + bwd 5 (FlashAttention accounting) = 3.5 x the forward
        r["engine_fwd_bwd_tflops_algorithmic"] = 3.5 * flops_fwd / (r["engine_fwd_bwd_ms"] * 1e-3) / 1e12
        out[str(dt).replace("torch.", "")] = {k2: round(v2, 4) for k2, v2 in r.items()}
        print(json.dumps({str(dt): out[str(dt).replace("torch.", "")]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
