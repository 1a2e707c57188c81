"""Where does the bf16 mode's error at the headline config come from?

Runs DGCNN(emb 1024) train fwd+bwd at B 32, N 1024, k 20 in bf16 mode and
compares against the fp64 oracle routed by the engine's decisions (on the GPU
in float64): the error of each block's output (the concat buffer) and of the
final output/gradients, for the product path and for variants selected by
``--variant``. Diagnostic only (tools/), not a test.
"""
import argparse
import os
import sys
import types

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]

from dgx import edgeconv as E  # noqa: E402
from dgx import precision, synth  # noqa: E402
from models.dgcnn import DGCNN  # noqa: E402
from oracle import reference as R  # noqa: E402


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--emb", type=int, default=1024)
    ap.add_argument("--z32", action="store_true", help="store conv5's Z in fp32 instead of bf16")
    ap.add_argument("--wexact", choices=["none", "edge", "conv5", "both"], default="none",
                    help="forward GEMMs with the fp32 (unrounded) weight: emulates a hi+lo bf16 weight split")
    a = ap.parse_args()
    from dgx import gemm as G0
    if a.wexact != "none":
        orig_prep_many, orig_prep_one, orig_lds = G0.prep_weights, G0.prep_weight, G0.lds_xwt
        from dgx.edgeconv import split_weight

        def tag(nt, w, rows, cols, stacked):
            nt.w32 = split_weight(w, cols, rows) if stacked else w.reshape(rows, cols)
            return nt

        def prep_weights(jobs):
            out = orig_prep_many(jobs)
            res = []
            for (w, r, c, st), (nt, tn) in zip(jobs, out):
                want = (st and a.wexact in ("edge", "both")) or (not st and a.wexact in ("conv5", "both"))
                res.append((tag(nt, w, r, c, st) if want else nt, tn))
            return res

        def lds_xwt(x16, w16, *args, **kw):
            if hasattr(w16, "w32") and not args and not kw.get("accumulate") and kw.get("addend") is None:
                z = torch.mm(x16.float(), w16.w32.t())
                if kw.get("stats"):
                    part = torch.stack([z.sum(0), (z * z).sum(0)]).unsqueeze(0).contiguous()
                    return (z.to(torch.bfloat16) if kw.get("out_bf16") else z), part
                return z
            return orig_lds(x16, w16, *args, **kw)

        class _GE:
            def __getattr__(self, n):
                return getattr(G0, n)
        ge = _GE()
        ge.prep_weights = prep_weights
        ge.lds_xwt = lds_xwt
        import dgx.pointconv as P0
        import models.dgcnn as MD
        E.G = ge
        P0.G = ge
        MD._gemm = ge
    if a.z32:
        from dgx import pointconv as P
        G = P.G
        orig = G.lds_xwt

        class _G:
            def __getattr__(self, n):
                return getattr(G, n)

            @staticmethod
            def lds_xwt(*args, **kw):
                kw["out_bf16"] = False
                return orig(*args, **kw)
        P.G = _G()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    k = 20
    m = DGCNN(types.SimpleNamespace(emb_dim=a.emb, k=k))
    init = {n: t.detach().clone() for n, t in m.state_dict().items()}
    m = m.to(dev).train()
    pts = synth.cube_clouds(a.B, a.N, 0)
    x = torch.from_numpy(pts).to(dev).permute(0, 2, 1)
    gout = torch.from_numpy(synth.uniform(1234, (a.B, a.emb, a.N)) - 0.5).float().to(dev)
    precision.set("bf16")
    E.set_debug_capture({})
    y = m(x)
    y.backward(gout)
    cap = E.debug_capture()
    E.set_debug_capture(None)
    precision.set("fp32")
    dec = [(i.long(), ar, z) for (i, ar, z) in (cap[("fwd", l)] for l in range(4))]
    params = {n: (t.to(dev).double() if t.is_floating_point() else t.to(dev)) for n, t in init.items()}
    for n, t in params.items():
        if t.is_floating_point() and "running" not in n:
            t.requires_grad_(True)
    xd = torch.from_numpy(pts).to(dev).double().permute(0, 2, 1)
    h, feats = xd, []
    for i in range(1, 5):
        idx, arg, zpos = dec[i - 1]
        h, _ = R.edgeconv_block_routed(h, params[f"conv{i}.0.weight"], R._bn(params, f"conv{i}.1"), idx, arg, zpos)
        feats.append(h)
    z = F.conv2d(torch.cat(feats, 1).unsqueeze(-1), params["conv5.0.weight"])
    zb = F.batch_norm(z, None, None, params["conv5.1.weight"], params["conv5.1.bias"], True, 0.1, 1e-5)
    zb = zb.view(a.B, -1, a.N)
    ref = torch.where(y.detach() > 0, zb, 0.2 * zb)
    ref.backward(gout.double())
    print("out", round(rel(y.detach(), ref.detach()), 5))
    precision.set("bf16")
    with torch.no_grad():
        xc = E.edgeconv_stack(x, k, m.edge_blocks()).view(a.B, a.N, -1)
    precision.set("fp32")
    off = 0
    for i, f in enumerate(feats):
        c = f.shape[1]
        print("block%d" % (i + 1), round(rel(xc[:, :, off:off + c].permute(0, 2, 1), f.detach()), 5))
        off += c
    zz = z.view(a.B, -1, a.N)
    mu = zz.mean(dim=(0, 2))
    sd = zz.std(dim=(0, 2))
    print("conv5 Z: mean|mu|/sd %.3f, max|mu|/sd %.3f" % (float((mu.abs() / sd).mean()), float((mu.abs() / sd).max())))
    for n, p in m.named_parameters():
        print(n, round(rel(p.grad, params[n].grad), 5))


if __name__ == "__main__":
    main()
