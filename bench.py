"""Headline benchmark (BASELINE.json metric):
    "point-clouds/sec + EdgeConv fwd+bwd ms at B=32 N=1024 k=20, 1/2/4/8 MI355X"

One step = DGCNN(emb=1024, k=20) forward + backward + SGD update on one batch of
32 synthetic clouds of 1024 points per GPU (BASELINE configs[1], "cfg2"), inputs
resident in HBM. N GPUs: one process per GPU (torchrun), DDP gradient
all-reduce over RCCL, weak scaling (32 clouds per GPU).

Prints ONE JSON line on rank 0 (contract in the task statement): whole-job
clouds/s, plus
  roofline      the kNN selection kernel (the engine's hot kernel) timed with
                HIP events on its own stream inside the timed region;
  cpu_baseline  the reference's CPU path (oracle/reference.py restatement,
                pinned by tests/golden) on a bounded sample, rank 0, N=1 only;
  edgeconv_fwd_bwd_ms  the 4-block EdgeConv chain alone (fwd+bwd), and
  torch_eager_gpu      the reference op sequence in stock PyTorch-ROCm on the
                       same GPU (the ">=10x" denominator), N=1 only.
"""
import argparse
import glob
import json
import os
import sys
import time
import types

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dgcnn.pytorch_amd"))

from dgx import gemm as dgx_gemm  # noqa: E402
from dgx import ops as dgx_ops  # noqa: E402
from dgx import precision as dgx_prec  # noqa: E402
from dgx import synth  # noqa: E402
from dgx.edgeconv import edgeconv_stack  # noqa: E402
from models.dgcnn import DGCNN  # noqa: E402

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 vector = f32 MFMA peak
PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)

METRIC = "point-clouds/sec + EdgeConv fwd+bwd ms at B=32 N=1024 k=20, 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", choices=["cfg2", "cfg3", "cfg5"], default="cfg2",
                   help="BASELINE.json configs: cfg2 N1024 k20 B32 (headline), cfg3 N2048 k40 B32, "
                        "cfg5 N4096 k20 B24 (S3DIS block size; DGCNN on xyz)")
    p.add_argument("--batch", type=int, default=None, help="clouds per GPU (default: the config's)")
    p.add_argument("--points", type=int, default=None)
    p.add_argument("--k", type=int, default=None)
    p.add_argument("--emb", type=int, default=1024)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-eager-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=8, help="clouds in the CPU baseline sample")
    p.add_argument("--precision", choices=["bf16", "fp32"], default="bf16",
                   help="GEMM operand precision (BASELINE cfg2 is bf16; fp32 is the parity mode)")
    p.add_argument("--no-fp32-leg", action="store_true", help="skip the extra fp32-mode timing")
    p.add_argument("--no-edgeconv-leg", action="store_true", help="skip the EdgeConv-only fwd+bwd timing")
    p.add_argument("--no-posemb-leg", action="store_true",
                   help="skip the PositionEmbedding edge-MLP timing (partseg geometry)")
    p.add_argument("--sync-bn", action="store_true",
                   help="N>1: SyncBatchNorm (global-batch BN statistics, main_partseg_dist.py:189) instead of "
                        "per-replica BN (main_cls.py:62 DataParallel semantics)")
    a = p.parse_args()
    preset = {"cfg2": (32, 1024, 20), "cfg3": (32, 2048, 40), "cfg5": (24, 4096, 20)}[a.config]
    a.batch = a.batch or preset[0]
    a.points = a.points or preset[1]
    a.k = a.k or preset[2]
    return a


_GRADS = {}


def upstream_grad(shape, dev):
    """The loss head's gradient w.r.t. DGCNN's (B, emb, N) output: a fixed
    random tensor, made once outside every timed region. The reference DGCNN
    is an embedding net with no loss of its own (models/dgcnn.py:80-103); all
    three legs (engine, eager PyTorch, CPU) back-propagate the same kind of
    dense upstream gradient."""
    key = (tuple(shape), str(dev))
    if key not in _GRADS:
        g = torch.Generator().manual_seed(1234)
        _GRADS[key] = (torch.rand(tuple(shape), generator=g) - 0.5).to(dev)
    return _GRADS[key]


def reduce_elapsed(elapsed, world, dev):
    """The job's time for the timed region: the slowest rank's (max over ranks)."""
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sync_all(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()


def timed_region(step, steps, world):
    sync_all(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync_all(world)
    return time.perf_counter() - t0


def edgeconv_only_ms(model, x, reps=10):
    """4-block EdgeConv chain fwd+bwd alone (the metric's second number)."""
    blocks = model.edge_blocks()
    g = None

    def run():
        nonlocal g
        out = edgeconv_stack(x, model.k, blocks, True)
        if g is None:
            g = torch.randn_like(out)
        out.backward(g)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def eager_reference_step_ms(x, k, emb, reps=5):
    """The reference's DGCNN op sequence (models/dgcnn.py:6-103: matmul, sum,
    topk, index gather, repeat, cat, permute, conv, BN, LeakyReLU, max) in stock
    PyTorch-ROCm eager on this GPU: the single-GPU denominator of the >=10x goal."""
    import torch.nn as nn
    import torch.nn.functional as F
    dev = x.device

    def gf(h):
        B, C, N = h.shape
        inner = -2 * torch.matmul(h.transpose(2, 1).contiguous(), h)
        hh = torch.sum(h ** 2, dim=1, keepdim=True)
        idx = (-hh - inner - hh.transpose(2, 1).contiguous()).topk(k=k, dim=-1)[1]
        idx = (idx + torch.arange(B, device=dev).view(-1, 1, 1) * N).view(-1)
        rows = h.transpose(2, 1).contiguous()
        nb = rows.view(B * N, -1)[idx, :].view(B, N, k, C)
        ctr = rows.view(B, N, 1, C).repeat(1, 1, k, 1)
        return torch.cat((nb, ctr), dim=3).permute(0, 3, 1, 2).contiguous()

    torch.manual_seed(0)
    widths = (64, 64, 128, 256)
    convs, c = [], 3
    for w in widths:
        convs.append(nn.Sequential(nn.Conv2d(2 * c, w, 1, bias=False), nn.BatchNorm2d(w),
                                   nn.LeakyReLU(0.2, inplace=True)).to(dev))
        c = w
    c5 = nn.Sequential(nn.Conv2d(512, emb, 1, bias=False), nn.BatchNorm2d(emb),
                       nn.LeakyReLU(0.2, inplace=True)).to(dev)

    def step():
        h, feats = x, []
        for m in convs:
            h = m(gf(h)).max(dim=-1, keepdim=False)[0]
            feats.append(h)
        y = c5(torch.cat(feats, dim=1).unsqueeze(-1)).view(x.shape[0], -1, x.shape[2])
        y.backward(upstream_grad(y.shape, dev))
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    del F
    return (time.perf_counter() - t0) / reps * 1e3


def posemb_edge_leg(dev, B=32, N=2048, k=40, reps=5):
    """a6: PositionEmbedding's edge stage (reference models/layers.py:45-52:
    get_graph_feature -> conv1 -> conv2 -> max over k), fwd+bwd, at the partseg
    geometry (BASELINE cfg4 per GPU: B 32, N 2048, k 40): the engine's fused op
    (dgx.edgemlp) next to the reference's op sequence in PyTorch-ROCm eager."""
    import torch.nn as nn
    from dgx.edgemlp import edge_mlp2
    torch.manual_seed(1)

    def blocks():
        return (nn.Sequential(nn.Conv2d(6, 64, 1, bias=False), nn.BatchNorm2d(64), nn.LeakyReLU(0.2)).to(dev),
                nn.Sequential(nn.Conv2d(64, 128, 1, bias=False), nn.BatchNorm2d(128), nn.LeakyReLU(0.2)).to(dev))
    x = (torch.rand(B, 3, N, device=dev) * 2 - 1).requires_grad_(True)
    g = torch.randn(B, 128, N, device=dev)
    c1, c2 = blocks()

    def engine():
        edge_mlp2(x, k, c1, c2, True).backward(g)

    def eager():
        B_, C, N_ = x.shape
        inner = -2 * torch.matmul(x.transpose(2, 1).contiguous(), x)
        xx = torch.sum(x ** 2, dim=1, keepdim=True)
        idx = (-xx - inner - xx.transpose(2, 1).contiguous()).topk(k=k, dim=-1)[1]
        idx = (idx + torch.arange(B_, device=dev).view(-1, 1, 1) * N_).view(-1)
        rows = x.transpose(2, 1).contiguous()
        nb = rows.view(B_ * N_, -1)[idx, :].view(B_, N_, k, C)
        ctr = rows.view(B_, N_, 1, C).repeat(1, 1, k, 1)
        e = torch.cat((nb, ctr), dim=3).permute(0, 3, 1, 2).contiguous()
        e1, e2 = eager_blocks
        e2(e1(e)).max(dim=-1)[0].backward(g)
    eager_blocks = blocks()

    def ms(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3
    out = {"config": f"B={B} N={N} k={k}, conv 6->64->128, train-mode BN, fwd+bwd"}
    out["engine_ms"] = round(ms(engine), 3)
    try:
        out["torch_eager_gpu_ms"] = round(ms(eager), 2)
        out["speedup"] = round(out["torch_eager_gpu_ms"] / out["engine_ms"], 2)
    except RuntimeError as e:
        out["torch_eager_gpu_ms"] = {"error": str(e)[:200]}
    return out


def cpu_baseline(args):
    """oracle/reference.py (torch-CPU restatement of the reference, golden-pinned)
    timed on the host cores for DGCNN(emb) fwd+bwd on a bounded sample."""
    sys.path.insert(0, REPO)
    from oracle import reference as R
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    model = DGCNN(types.SimpleNamespace(emb_dim=args.emb, k=args.k))  # same init/param layout
    params = {n: t.detach().clone() for n, t in model.state_dict().items()}
    for n, t in params.items():
        if t.is_floating_point() and "running" not in n:
            t.requires_grad_(True)
    Bs = args.cpu_sample
    x = torch.from_numpy(synth.cube_clouds(Bs, args.points, 0)).permute(0, 2, 1)

    def step():
        y, _ = R.dgcnn(x, args.k, params, training=True)
        y.backward(upstream_grad(y.shape, torch.device("cpu")))
    step()
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(Bs / med, 3), "unit": "clouds/s", "cores": threads, "kind": "port",
            "sample": f"oracle/reference.py DGCNN(emb={args.emb}) train fwd+bwd, {Bs} clouds x {args.points} pts, "
                      f"k={args.k}, median of 3 after 1 warm-up, torch CPU {threads} threads",
            "ms_per_step_sample": round(med * 1e3, 1)}


def latest_pmc_traffic():
    """HBM bytes per kNN launch from the committed rocprofv3 PMC summary, if any."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*knn_pmc*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    dgx_prec.set(args.precision)
    torch.manual_seed(0)
    model = DGCNN(types.SimpleNamespace(emb_dim=args.emb, k=args.k)).to(dev).train()
    net = model
    if world > 1:
        if args.sync_bn:
            model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
        net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local])
    try:  # one fused kernel for the whole parameter list (same math as the foreach form)
        opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, fused=True)
    except (RuntimeError, TypeError, ValueError):
        opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    pts = torch.from_numpy(synth.cube_clouds(args.batch, args.points, seed=rank)).to(dev)
    x = pts.permute(0, 2, 1)  # (B,3,N) view, as main_cls.py:91 feeds the model

    gy = upstream_grad((args.batch, args.emb, args.points), dev)

    def step():
        opt.zero_grad(set_to_none=True)
        y = net(x)
        y.backward(gy)
        opt.step()

    for _ in range(args.warmup):
        step()
    # headline: the timed region runs uninstrumented
    elapsed = timed_region(step, args.steps, world)
    # roofline / MFMA: the same K steps again with HIP events around every kNN
    # selection and GEMM launch (on their launch stream); events perturb the
    # step slightly, so this region is reported separately
    timing, gtiming = [], []
    dgx_ops.set_knn_timing(timing)
    dgx_gemm.set_timing(gtiming)
    elapsed_inst = timed_region(step, args.steps, world)
    dgx_ops.set_knn_timing(None)
    dgx_gemm.set_timing(None)
    elapsed = reduce_elapsed(elapsed, world, dev)
    elapsed_inst = reduce_elapsed(elapsed_inst, world, dev)

    knn_ms = [e0.elapsed_time(e1) for (e0, e1, _, _) in timing]
    knn_flops = [f for (_, _, f, _) in timing]
    launches = max(1, len(knn_ms))
    avg_ms = sum(knn_ms) / launches
    avg_flops = sum(knn_flops) / launches
    achieved = avg_flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    per_layer = {}
    for (ms, (_, _, _, shape)) in zip(knn_ms, timing):
        per_layer.setdefault(f"C{shape[1]}", []).append(ms)
    per_layer = {c: round(sum(v) / len(v), 4) for c, v in per_layer.items()}

    g_ms = sum(e0.elapsed_time(e1) for (e0, e1, _, _) in gtiming)
    g_flops = sum(f for (_, _, f, _) in gtiming)
    by_tag = {}
    for (e0, e1, f, tg) in gtiming:
        if tg is not None:
            ms, fl, n = by_tag.get(tg, (0.0, 0.0, 0))
            by_tag[tg] = (ms + e0.elapsed_time(e1), fl + f, n + 1)
    peak_g = PEAK_BF16_TFLOPS if args.precision == "bf16" else PEAK_FP32_TFLOPS
    conv5 = {tg: {"avg_launch_ms": round(ms / n, 4), "flops_per_launch": fl / n,
                  "achieved": round(fl / (ms * 1e-3) / 1e12, 1), "frac": round(fl / (ms * 1e-3) / 1e12 / peak_g, 4)}
             for tg, (ms, fl, n) in by_tag.items() if ms > 0}
    result = {
        "metric": METRIC,
        "value": round(args.batch * world * args.steps / elapsed, 2),
        "unit": "clouds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (splitmix64 uniform-cube clouds, random-init weights, fixed random upstream gradient)",
        "config": {"workload": f"DGCNN(emb={args.emb},k={args.k}) train step fwd+bwd+SGD, {args.config}",
                   "model": "DGCNN", "global_batch": args.batch * world, "points": args.points,
                   "seq_len": args.points, "k": args.k, "emb_dim": args.emb,
                   "parallelism": f"dp{world}" + ("+syncbn" if (args.sync_bn and world > 1) else "")},
        "roofline": {"kernel": "knn_kernel (fused fp32 Gram on MFMA + top-k)", "bound": "mfma",
                     "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                     "traffic": latest_pmc_traffic(),
                     "avg_launch_ms": round(avg_ms, 4), "algorithmic_flops_per_launch": avg_flops,
                     "launches_timed": len(knn_ms), "knn_ms_by_layer": per_layer,
                     "timed_region": "second K-step region with HIP events (ms_per_step %.3f)"
                                     % (elapsed_inst / args.steps * 1e3)},
        # the Conv(1x1) GEMMs of the chain and conv5 (fwd + dX + dW) on the bf16 MFMA.
        # Every GEMM launch is bracketed by HIP events (~20 us of marker overhead each
        # on this stack), so the all-GEMM sum is an upper bound of their time; the
        # three conv5 GEMMs (34 GFLOP each) are the per-kernel MFMA utilisation.
        "mfma_gemm": {"kernels": "gemm_lds_kernel / gemm_bf16_kernel (csrc/gemm.hip)",
                      "flops_per_step": g_flops / max(1, args.steps),
                      "event_bracketed_ms_per_step": round(g_ms / max(1, args.steps), 4),
                      "peak": peak_g, "unit": "TFLOP/s", "conv5": conv5},
    }
    if args.precision != "fp32" and not args.no_fp32_leg:
        dgx_prec.set("fp32")  # same model, parity-mode GEMMs
        for _ in range(2):
            step()
        el32 = timed_region(step, args.steps, world)
        el32 = reduce_elapsed(el32, world, dev)
        result["fp32_mode"] = {"ms_per_step": round(el32 / args.steps * 1e3, 3),
                               "value": round(args.batch * world * args.steps / el32, 2)}
        dgx_prec.set(args.precision)
    if rank == 0 and world == 1:
        if not args.no_edgeconv_leg:
            result["edgeconv_fwd_bwd_ms"] = round(edgeconv_only_ms(model, x), 3)
        if not args.no_posemb_leg:
            result["posemb_edge_mlp"] = posemb_edge_leg(dev)
        if not args.no_eager_baseline:
            try:
                ms = eager_reference_step_ms(x, args.k, args.emb)
                result["torch_eager_gpu"] = {"ms_per_step": round(ms, 2),
                                             "clouds_per_s": round(args.batch / ms * 1e3, 2),
                                             "speedup": round(ms / result["ms_per_step"], 2)}
            except RuntimeError as e:  # e.g. out of memory: report, don't hide
                result["torch_eager_gpu"] = {"error": str(e)[:200]}
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
