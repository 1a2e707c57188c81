"""A/B bit comparison of two libdgx builds: `python tools/ab_bitcmp.py OUT.pt`
runs one DGCNN train step (cfg2 geometry, bf16 and fp32 modes) with the build
DGX_LIB names and saves output, gradients and BN buffers; `--compare A.pt B.pt`
reports every tensor that differs."""
import sys
import types

import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "dgcnn.pytorch_amd"))


def run(path):
    from dgx import precision as prec, synth
    from models.dgcnn import DGCNN
    res = {}
    for mode in ("bf16", "fp32"):
        torch.manual_seed(1)
        m = DGCNN(types.SimpleNamespace(emb_dim=1024, k=20, in_dims=3)).cuda().train()
        x = torch.from_numpy(synth.cube_clouds(8, 1024, 3)).cuda().permute(0, 2, 1)
        g = torch.randn((8, 1024, 1024), device="cuda", generator=torch.Generator("cuda").manual_seed(2))
        with prec.mode(mode):
            y = m(x)
            y.backward(g)
        res[f"{mode}.y"] = y.detach().cpu()
        for n, p in m.named_parameters():
            res[f"{mode}.grad.{n}"] = p.grad.cpu()
        for n, b in m.named_buffers():
            res[f"{mode}.buf.{n}"] = b.cpu()
    torch.save(res, path)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = [n for n in A if not torch.equal(A[n], B[n])]
    print(f"{len(A)} tensors, {len(bad)} differ" + (": " + ", ".join(bad[:20]) if bad else ""))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
