"""A/B timing of the cfg2 train step (bench.py's step: DGCNN emb 1024, B 32,
N 1024, k 20, bf16, fwd + bwd + SGD) under module-attribute switches,
interleaved A, B, A, B ... so box drift hits every variant alike.
  python tools/ab_step.py "dgx.edgeconv:OVERLAP_DW=0" "dgx.edgeconv:OVERLAP_DW=1" [--rounds 5 --steps 20]
A variant is a comma-separated list of module:ATTR=int assignments ("" = as shipped)."""
import argparse
import importlib
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "dgcnn.pytorch_amd")):
    sys.path.insert(0, p)


_DEFAULTS = {}


def apply(spec, all_specs=()):
    """Set the variant's switches; every switch named by any variant is first
    reset to its shipped value (so "" really is the shipped configuration)."""
    for sp in all_specs:
        for item in filter(None, sp.split(",")):
            mod, rest = item.split(":")
            attr = rest.split("=")[0]
            m = importlib.import_module(mod)
            _DEFAULTS.setdefault((mod, attr), getattr(m, attr))
    for (mod, attr), val in _DEFAULTS.items():
        setattr(importlib.import_module(mod), attr, val)
    for item in filter(None, spec.split(",")):
        mod, rest = item.split(":")
        attr, val = rest.split("=")
        setattr(importlib.import_module(mod), attr, type(getattr(importlib.import_module(mod), attr))(int(val)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--points", type=int, default=1024)
    ap.add_argument("--graph", action="store_true", help="time HIP-graph replays (one capture per variant)")
    a = ap.parse_args()
    import torch

    import bench
    from dgx import precision
    from models.dgcnn import DGCNN
    dev = torch.device("cuda:0")
    precision.set("bf16")
    torch.manual_seed(0)
    model = DGCNN(types.SimpleNamespace(emb_dim=1024, k=20)).to(dev).train()
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, fused=True)
    bargs = bench.parse(["--batch", str(a.batch), "--points", str(a.points)])
    x = torch.from_numpy(bench.make_input(bargs, a.batch, seed=0)).to(dev).permute(0, 2, 1)
    gy = bench.upstream_grad((a.batch, 1024, a.points), dev)

    def step():
        opt.zero_grad(set_to_none=True)
        model(x).backward(gy)
        opt.step()

    res = {v: [] for v in a.variants}
    runs = {}
    for v in a.variants:  # warm every variant (and capture its graph)
        apply(v, a.variants)
        for _ in range(5):
            step()
        runs[v] = step
        if a.graph:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                step()
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            opt.zero_grad(set_to_none=True)
            with torch.cuda.graph(g):
                model(x).backward(gy)
                opt.step()
            runs[v] = g.replay
    for r in range(a.rounds):
        for v in a.variants:
            apply(v, a.variants)
            step = runs[v]
            step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                step()
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.steps)
    for v, ms in res.items():
        ms = sorted(ms)
        print(f"{v or '(shipped)':60s} median {ms[len(ms) // 2]:.4f} ms/step  min {ms[0]:.4f}  all "
              + " ".join(f"{m:.3f}" for m in res[v]), flush=True)


if __name__ == "__main__":
    main()
