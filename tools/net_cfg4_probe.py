"""Probe: Net at cfg4 geometry — per-parameter gradient error of the engine run
and of the stock fp32 restatement (same routing) against the stock fp64
restatement, to separate engine error from the problem's fp32 conditioning.
Usage: python tools/net_cfg4_probe.py [--amp] [--stock-attn]"""
import argparse
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd"), os.path.join(REPO, "tests")]

import dgx.edgeconv as E  # noqa: E402
import oracle  # noqa: E402
from conftest import edge_mlp_decisions, rel_err  # noqa: E402
from dgx import synth  # noqa: E402
from models.model_partseg import Net, compute_hog_1x1  # noqa: E402
from oracle.partseg import net_routed, stock_copy  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--amp", action="store_true")
ap.add_argument("--stock-attn", action="store_true")
ap.add_argument("--B", type=int, default=2)
a = ap.parse_args()
cuda = torch.device("cuda:0")
B, N, k, emb = a.B, 2048, 40, 512
args = types.SimpleNamespace(k=k, emb_dim=emb, n_heads=4, n_blocks=1, ff_dims=512, dropout=0.0, nclasses=50)
torch.manual_seed(17)
net = Net(args)
net64 = stock_copy(net).double().to(cuda).train()
net32 = stock_copy(net).to(cuda).train()
if a.stock_attn:
    net = stock_copy(net)
net = net.to(cuda).train()
pts = synth.cube_clouds(B, N, 170)
src = torch.from_numpy(pts).to(cuda).permute(0, 2, 1).contiguous()
lbl = torch.nn.functional.one_hot(torch.arange(B) * 5 % 16, 16).float().to(cuda)
gout = torch.from_numpy(synth.uniform(171, (B, 50, N)) - 0.5).float().to(cuda)
seen = {}
hooks = [net.emb_nn.register_forward_hook(lambda m, i, o: seen.__setitem__("emb", o.detach())),
         net.pos_mlp[0].conv3.register_forward_hook(lambda m, i, o: seen.__setitem__("t3", o.detach()))]
E.set_debug_capture({})
with torch.autocast("cuda", dtype=torch.float16, enabled=a.amp):
    out = net(src, lbl)
out.float().backward(gout)
cap = E.debug_capture()
E.set_debug_capture(None)
dgcnn_dec = [(i.long(), aa, z) for (i, aa, z) in (cap[("fwd", l)] for l in range(4))]
zpos1, arg2, zpos2, _ = edge_mlp_decisions(cap, B, N, k, net.pos_mlp[0].conv2[0].weight)
eidx = cap["emlp"]["idx"].view(B, N, k).long()
argmax_n = seen["t3"].max(dim=-1)[1]
hog = compute_hog_1x1(src, k)
res = {}
for name, m, dt in (("f64", net64, torch.float64), ("f32", net32, torch.float32)):
    r, _ = net_routed(m, src.to(dt), lbl.to(dt), dgcnn_dec, seen["emb"] > 0, (eidx, zpos1, arg2, zpos2), hog.to(dt),
                      argmax_n)
    r.backward(gout.to(dt))
    res[name] = (r.detach(), dict(m.named_parameters()))
gscale = max(float(p.grad.abs().max()) for p in res["f64"][1].values())
print("out: engine", rel_err(out.detach().float().cpu(), res["f64"][0].cpu()), "stock f32",
      rel_err(res["f32"][0].cpu(), res["f64"][0].cpu()))
rows = []
for n, p in net.named_parameters():
    g64 = res["f64"][1][n].grad.cpu()
    g32 = res["f32"][1][n].grad.cpu()
    den = max(float(g64.abs().max()), 1e-30)
    rows.append((n, rel_err(p.grad.float().cpu(), g64), rel_err(g32, g64), den / gscale))
rows.sort(key=lambda r: -r[1])
for n, e, e32, sc in rows[:40]:
    print(f"{n:50s} engine {e:.2e}  stock-f32 {e32:.2e}  |g|max/gscale {sc:.1e}")
