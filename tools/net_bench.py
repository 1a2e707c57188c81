"""Net (partseg) train step under fp16 autocast as main_partseg_dist.py runs it,
with the engine attention (f2) and, for comparison, the same weights on stock
PyTorch attention (every attention module switched back to
nn.MultiheadAttention).

  python tools/net_bench.py [--batch 8] [--points 2048] [--k 40]
"""
import argparse
import json
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--points", type=int, default=2048)
    ap.add_argument("--k", type=int, default=40)
    ap.add_argument("--emb", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from dgx import synth
    from dgx.attention import EngineMultiheadAttention
    from models.model_partseg import Net
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    args = types.SimpleNamespace(k=a.k, emb_dim=a.emb, n_heads=4, n_blocks=1, ff_dims=512, dropout=0.5, nclasses=50)
    net = Net(args).to(dev).train()
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
    scaler = torch.amp.GradScaler("cuda")
    src = torch.from_numpy(synth.cube_clouds(a.batch, a.points, 0)).to(dev).permute(0, 2, 1).contiguous()
    lbl = torch.nn.functional.one_hot(torch.arange(a.batch) % 16, 16).float().to(dev)
    target = torch.randint(0, 50, (a.batch, a.points), device=dev)
    mhas = [m for m in net.modules() if isinstance(m, torch.nn.MultiheadAttention)]

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            loss = torch.nn.functional.cross_entropy(net(src, lbl).float(), target)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()

    def timed():
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.reps * 1e3

    out = {"config": vars(a)}
    out["engine_attention_ms"] = round(timed(), 2)
    for m in mhas:
        m.__class__ = torch.nn.MultiheadAttention
    out["stock_attention_ms"] = round(timed(), 2)
    for m in mhas:
        m.__class__ = EngineMultiheadAttention
    out["speedup"] = round(out["stock_attention_ms"] / out["engine_attention_ms"], 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
