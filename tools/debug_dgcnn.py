"""Per-layer error breakdown of the fused DGCNN vs an fp64 oracle run with the
GPU's own neighbour sets."""
import os, sys, types
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd"), os.path.join(REPO, "tests")]
from conftest import load_golden, rel_err  # noqa
from oracle import reference as R  # noqa
from models.dgcnn import DGCNN, knn  # noqa
from dgx.edgeconv import edgeconv_stack  # noqa

g = load_golden("dgcnn_small.npz")
dev = torch.device("cuda:0")
m = DGCNN(types.SimpleNamespace(emb_dim=64, k=10))
m.load_state_dict({n[5:]: torch.from_numpy(g[n]) for n in g.files if n.startswith("init.")})
m = m.to(dev).train()
x = torch.from_numpy(g["x"]).to(dev)
B, _, N = x.shape
# GPU features and per-layer idx
with torch.no_grad():
    feats = edgeconv_stack(x, 10, m.edge_blocks(), True)
f = feats.view(B, N, -1).permute(0, 2, 1).contiguous().cpu()
idx = [knn(x, 10).cpu()]
off = 0
for w in (64, 64, 128):
    idx.append(knn(f[:, off:off + w].contiguous().to(dev), 10).cpu())
    off += w
# fresh model for grads
m2 = DGCNN(types.SimpleNamespace(emb_dim=64, k=10))
m2.load_state_dict({n[5:]: torch.from_numpy(g[n]) for n in g.files if n.startswith("init.")})
m2 = m2.to(dev).train()
y = m2(x)
y.backward(torch.from_numpy(g["gout"]).to(dev))
params = {n[5:]: torch.from_numpy(g[n].copy()).double() if g[n].dtype == np.float32 else torch.from_numpy(g[n].copy())
          for n in g.files if n.startswith("init.")}
for n, t in params.items():
    if t.is_floating_point() and "running" not in n:
        t.requires_grad_(True)
y64, _ = R.dgcnn(torch.from_numpy(g["x"]).double(), 10, params, training=True, idx_list=idx)
y64.backward(torch.from_numpy(g["gout"]).double())
print("out vs fp64: %.2e   golden vs fp64: %.2e" % (rel_err(y.detach().cpu(), y64.detach()), rel_err(g["out"], y64.detach())))
# per-layer features
h = torch.from_numpy(g["x"]).double()
off = 0
for i, w in enumerate((64, 64, 128, 256), start=1):
    bn = R._bn({k: v.detach() for k, v in params.items()}, f"conv{i}.1")
    bn = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in bn.items()}
    h = R.edgeconv_block(h, 10, params[f"conv{i}.0.weight"].detach(), bn, True, idx=idx[i - 1])
    print(f"x{i} vs fp64: %.2e" % rel_err(f[:, off:off + w], h))
    off += w
for n, p in m2.named_parameters():
    print("%-16s gpu %.2e   golden %.2e" % (n, rel_err(p.grad.cpu(), params[n].grad), rel_err(g["grad." + n], params[n].grad)))

# ---- capture block-4 internals and compare with fp64 autograd of the reference
import dgx.edgeconv as E  # noqa
E._debug = {}
m3 = DGCNN(types.SimpleNamespace(emb_dim=64, k=10))
m3.load_state_dict({n[5:]: torch.from_numpy(g[n]) for n in g.files if n.startswith("init.")})
m3 = m3.to(dev).train()
y3 = m3(x)
y3.backward(torch.from_numpy(g["gout"]).to(dev))
d4 = {k: v.cpu() for k, v in E._debug[3].items()}
dz = d4["dz"].double()
print("gpu dbeta4 from kernel vs sum(dz) recomputed: %.2e" % rel_err(d4["dbeta"], dz.sum(0)))
print("dbeta4 kernel vs fp64: %.2e ; sum(dz) vs fp64: %.2e" % (rel_err(d4["dbeta"], params["conv4.1.bias"].grad),
      rel_err(dz.sum(0), params["conv4.1.bias"].grad)))
part = d4["partials"].double()
print("partials sum vs kernel dbeta: %.2e" % rel_err(part[:, 0, :].sum(0), d4["dbeta"]))
print("nblk", part.shape, "M", dz.shape)

# fp64 reference: gradient w.r.t. x4 (output of block 4) and the dz at selected edges
h = torch.from_numpy(g["x"]).double()
feats64 = []
p64 = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in params.items()}
for i in range(1, 5):
    bn = R._bn(p64, f"conv{i}.1")
    bn = dict(bn)
    bn["running_mean"] = bn["running_mean"].clone(); bn["running_var"] = bn["running_var"].clone()
    h = R.edgeconv_block(h, 10, p64[f"conv{i}.0.weight"], bn, True, idx=idx[i - 1])
    h.retain_grad()
    feats64.append(h)
zz = torch.cat(feats64, 1).unsqueeze(-1)
o64 = R.conv_bn_lrelu(zz, p64["conv5.0.weight"], R._bn(p64, "conv5.1"), True).view(B, -1, N)
o64.backward(torch.from_numpy(g["gout"]).double())
dY4_ref = feats64[3].grad.permute(0, 2, 1).reshape(B * N, -1)
print("dY4 gpu vs fp64: %.2e" % rel_err(d4["dY"], dY4_ref))
dY3_ref = feats64[2].grad.permute(0, 2, 1).reshape(B * N, -1)
print("dY3(after add) gpu vs fp64: %.2e" % rel_err(E._debug[2]["dY"].cpu(), dY3_ref))
print("dbeta4 gpu", d4["dbeta"][:6].tolist())
print("dbeta4 ref", params["conv4.1.bias"].grad[:6].tolist())
print("dgamma4 gpu", d4["dgamma"][:4].tolist(), "ref", params["conv4.1.weight"].grad[:4].tolist())

# fp64 per-edge gradient of block 4's conv output -> reference dP, dQ
import torch.nn.functional as Fn  # noqa
h = torch.from_numpy(g["x"]).double()
p5 = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in params.items()}
feats5 = []
for i in range(1, 5):
    bn = dict(R._bn(p5, f"conv{i}.1"))
    bn["running_mean"] = bn["running_mean"].clone(); bn["running_var"] = bn["running_var"].clone()
    e = R.graph_feature(h, 10, idx=idx[i - 1])
    yconv = Fn.conv2d(e, p5[f"conv{i}.0.weight"])
    if i == 4:
        yconv.retain_grad(); y4 = yconv
    zb = Fn.batch_norm(yconv, bn["running_mean"], bn["running_var"], bn["weight"], bn["bias"], True, 0.1, 1e-5)
    if i == 4:
        zb.retain_grad(); zb4 = zb
    h = Fn.leaky_relu(zb, 0.2).max(dim=-1)[0]
    feats5.append(h)
zz = torch.cat(feats5, 1).unsqueeze(-1)
o5 = R.conv_bn_lrelu(zz, p5["conv5.0.weight"], R._bn(p5, "conv5.1"), True).view(B, -1, N)
o5.backward(torch.from_numpy(g["gout"]).double())
dy = y4.grad  # (B, Co, N, k)
Co = dy.shape[1]
dQ_ref = dy.sum(-1).permute(0, 2, 1).reshape(B * N, Co)
dP_ref = torch.zeros(B * N, Co, dtype=torch.float64)
gidx = (idx[3] + torch.arange(B).view(-1, 1, 1) * N).reshape(-1)
dP_ref.index_add_(0, gidx, dy.permute(0, 2, 3, 1).reshape(-1, Co))
dPQ = d4["dPQ"].double()
print("dP4 gpu vs fp64: %.2e   dQ4: %.2e" % (rel_err(dPQ[:, :Co], dP_ref), rel_err(dPQ[:, Co:], dQ_ref)))
err = (dPQ[:, :Co] - dP_ref).abs()
r, c = divmod(int(err.argmax()), Co)
print("worst dP at point", r, "ch", c, "gpu", float(dPQ[r, c]), "ref", float(dP_ref[r, c]))
indeg = torch.bincount(gidx, minlength=B * N)
print("indeg of worst", int(indeg[r]), "max indeg", int(indeg.max()))

# argmax flips in block 4: fp64 edge outputs vs the GPU's chosen argument
e4 = R.graph_feature(feats5[2].detach(), 10, idx=idx[3])            # (B, 2C, N, k) fp64 from fp64 x3
y4r = Fn.conv2d(e4, p5["conv4.0.weight"].detach())                   # (B, Co, N, k)
ref_arg = y4r.argmax(-1).permute(0, 2, 1).reshape(B * N, -1)
garg = d4["arg"].long()
flips = (ref_arg != garg)
print("block4 argmax flips:", int(flips.sum()), "of", flips.numel())
if flips.any():
    yv = y4r.permute(0, 2, 3, 1).reshape(B * N, 10, -1)
    r, c = torch.nonzero(flips)[0].tolist()
    top = yv[r, :, c]
    print("  values at flip (ref argmax %d, gpu %d):" % (ref_arg[r, c], garg[r, c]), float(top[ref_arg[r, c]]), float(top[garg[r, c]]))

# self-consistency of block 4 from the captured GPU intermediates (fp64 on CPU)
D = {k: v.cpu().double() if v.is_floating_point() else v.cpu() for k, v in E._debug[3].items()}
Co = D["dz"].shape[1]; k = 10; M = B * N
P, Q = D["PQ"][:, :Co], D["PQ"][:, Co:]
gi = (D["idx"].long() + torch.arange(B).view(-1, 1, 1) * N).reshape(M, k)
print("sumP consistent: %.2e" % rel_err(D["sumP"], P[gi].sum(1)))
print("PQ vs X W^T: %.2e" % rel_err(D["PQ"], D["X"] @ torch.cat([p5["conv4.0.weight"].detach().view(Co, -1)[:, :128], p5["conv4.0.weight"].detach().view(Co, -1)[:, 128:]], 0).t()))
a, c0, c1 = D["scale"], D["c0"], D["c1"]
dQ_cpu = a * D["dz"] + k * c0 + c1 * (D["sumP"] + k * Q)
print("dQ kernel vs formula: %.2e" % rel_err(D["dPQ"][:, Co:], dQ_cpu))
# dP via explicit edges
dP_cpu = torch.zeros(M, Co, dtype=torch.float64)
argsel = D["arg"].long()
for i in range(M):
    for kk in range(k):
        j = gi[i, kk]
        y = P[j] + Q[i]
        dye = c0 + c1 * y + a * D["dz"][i] * (argsel[i] == kk)
        dP_cpu[j] += dye
print("dP kernel vs formula: %.2e" % rel_err(D["dPQ"][:, :Co], dP_cpu))
print("dP formula vs fp64 ref: %.2e" % rel_err(dP_cpu, dP_ref))
rp, ed = D["rowptr"].long(), D["edges"].long()
deg = rp[1:] - rp[:-1]
print("CSR indeg matches idx:", bool((deg == torch.bincount(gi.reshape(-1), minlength=M)).all()), "total", int(rp[-1]))
ok = True
for j in range(M):
    es = sorted(((int(e) >> 6), int(e) & 63) for e in ed[rp[j]:rp[j + 1]])
    exp = sorted((i, kk) for i in range(M) for kk in range(k) if gi[i, kk] == j) if j < 3 else None
    if exp is not None and es != exp:
        ok = False
print("CSR lists (first 3 points) ok:", ok)
# BN stats consistency
yall = (P[gi] + Q[:, None, :])  # (M,k,Co)
mu = yall.mean((0, 1)); var = yall.var((0, 1), unbiased=False)
print("mean %.2e invstd %.2e" % (rel_err(D["mean"], mu), rel_err(D["invstd"], 1 / torch.sqrt(var + 1e-5))))

dzr = zb4.grad.permute(0, 2, 3, 1).reshape(M, k, Co)          # reference dL/dz per edge
nz = (dzr != 0).sum(1)
print("edges with nonzero dz per (i,o): min", int(nz.min()), "max", int(nz.max()))
dz_ref_sel = dzr.sum(1)
print("dz gpu vs ref (selected): %.2e" % rel_err(D["dz"], dz_ref_sel))
g1r = dzr.sum((0, 1)) / (M * k)
yhat = (y4r.permute(0, 2, 3, 1).reshape(M, k, Co) - D["mean"]) * D["invstd"]
g2r = (dzr * yhat).sum((0, 1)) / (M * k)
print("sum dz gpu(dbeta) vs ref: %.2e ; sum dz*yhat: %.2e" % (rel_err(D["dbeta"], g1r * M * k), rel_err(D["dgamma"], g2r * M * k)))
c0r = a * (-g1r + g2r * D["mean"] * D["invstd"]); c1r = -a * g2r * D["invstd"]
print("c0 %.2e c1 %.2e" % (rel_err(D["c0"], c0r), rel_err(D["c1"], c1r)))
dyr = y4.grad.permute(0, 2, 3, 1).reshape(M, k, Co)
ymine = P[gi] + Q[:, None, :]
dymine = c0 + c1 * ymine + a * D["dz"][:, None, :] * (argsel[:, None, :] == torch.arange(k).view(1, k, 1))
print("dy per edge mine vs ref: %.2e" % rel_err(dymine, dyr))
dyr2 = a * (dzr - g1r - ((ymine - D["mean"]) * D["invstd"]) * g2r)
print("dy textbook(ref dz) vs ref: %.2e" % rel_err(dyr2, dyr))
zsel = D["scale"] * D["ysel"] + D["shift"]
dz_check = D["dY"] * torch.where(zsel > 0, 1.0, 0.2)
print("dz kernel vs recompute from dY: %.2e" % rel_err(D["dz"], dz_check))
print("dz recompute vs ref: %.2e" % rel_err(dz_check, dz_ref_sel))
zr = zb4.detach().permute(0, 2, 3, 1).reshape(M, k, Co)
zr_sel = torch.gather(zr, 1, argsel[:, None, :]).squeeze(1)
print("z_sel gpu vs ref: %.2e ; mask disagreements: %d" % (rel_err(zsel, zr_sel), int(((zsel > 0) != (zr_sel > 0)).sum())))
dYr = dY4_ref
print("dY ref vs D: %.2e" % rel_err(D["dY"], dYr))
bad = (dz_check - dz_ref_sel).abs() > 1e-3 * dz_ref_sel.abs().max()
print("bad elements:", int(bad.sum()), "channels:", torch.nonzero(bad)[:5, 1].tolist(), "rows:", torch.nonzero(bad)[:5, 0].tolist())
