"""Print every parameter's rel err of the routed-oracle DGCNN parity check for
one (emb, N, k, B) case (debugging aid for tests/test_edgeconv_gpu.py)."""
import os
import sys
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd"), os.path.join(REPO, "tests")]
from conftest import rel_err  # noqa: E402
from oracle import reference as R  # noqa: E402
from test_edgeconv_gpu import Capture  # noqa: E402

emb, N, k, B = (int(v) for v in sys.argv[1:5])
from models.dgcnn import DGCNN  # noqa: E402
from dgx import synth  # noqa: E402
cuda = torch.device("cuda:0")
torch.manual_seed(emb + N)
m = DGCNN(types.SimpleNamespace(emb_dim=emb, k=k))
init = {n: t.detach().clone() for n, t in m.state_dict().items()}
m = m.to(cuda).train()
pts = synth.cube_clouds(B, N, 60 + N)
x = torch.from_numpy(pts).to(cuda).permute(0, 2, 1)
with Capture() as cap:
    y = m(x)
gout = torch.from_numpy(synth.uniform(61, tuple(y.shape)) - 0.5)
y.backward(gout.to(cuda))
decisions = [tuple(t.cpu() for t in cap[("fwd", l)]) for l in range(4)]
decisions = [(i.long(), a, z) for (i, a, z) in decisions]
params = {n: (t.double() if t.is_floating_point() else t) for n, t in init.items()}
for n, t in params.items():
    if t.is_floating_point() and "running" not in n:
        t.requires_grad_(True)
ref = R.dgcnn_routed(torch.from_numpy(pts).double().permute(0, 2, 1), params, decisions, y.detach().cpu() > 0)
ref.backward(gout.double())
print("y", rel_err(y.detach().cpu(), ref.detach()))
p32 = {n: (t.float().detach().requires_grad_(t.requires_grad) if t.is_floating_point() else t)
       for n, t in params.items()}
ref32 = R.dgcnn_routed(torch.from_numpy(pts).float().permute(0, 2, 1), p32, decisions, y.detach().cpu() > 0)
ref32.backward(gout.float())
for n, p in m.named_parameters():
    g64 = params[n].grad
    print(f"{n:18s} engine {rel_err(p.grad.cpu(), g64):.2e}  fp32-oracle {rel_err(p32[n].grad, g64):.2e}  "
          f"max|g| {float(g64.abs().max()):.3e}  |sum| {float(g64.sum()):.3e}")
for l in range(4):
    d = cap.get(l, {})
    print("layer", l, {kk: float(v.float().abs().max()) for kk, v in d.items() if kk in ("dz", "dPQ")})
