"""Headline benchmark (BASELINE.json metric):
    "point-clouds/sec + EdgeConv fwd+bwd ms at B=32 N=1024 k=20, 1/2/4/8 MI355X"

One step = DGCNN(emb=1024, k=20) forward + backward + SGD update on one batch of
synthetic clouds (BASELINE configs[1], "cfg2": 32 clouds of 1024 points per
GPU), inputs resident in HBM. The SGD update (lr 0.1, momentum 0.9, weight
decay 1e-4) is dgx.optim.SGD — torch.optim.SGD's update in one launch;
``--sgd fused`` runs torch's own fused kernel instead.

N GPUs: one process per GPU over RCCL (torch.distributed "nccl"), DDP gradient
all-reduce. ``python bench.py --gpus N`` with no WORLD_SIZE in the environment
starts the N ranks itself (torch.distributed.run as a child process, before
anything touches the GPU); under an outer torchrun it is one rank.
``--scaling weak`` (default): B clouds per GPU. ``--scaling strong``: the global
batch B is split over the ranks, B / world per GPU (main_partseg_dist.py:165).

Prints ONE JSON line on rank 0: whole-job clouds/s, plus
  roofline      the kNN selection kernel (the engine's largest kernel family):
                its launches bracketed by HIP events on their own stream in a
                second K-step region (only those launches, 8 events per step);
                HBM traffic per launch from the committed rocprofv3 PMC summary
                of this config (profiles/*_pmc_<config>.json), refused unless its
                kernel names match the kernels this build launches;
  cpu_baseline  the reference's CPU path (oracle/reference.py restatement,
                golden-pinned) for the same B-cloud batch on the host cores
                this job is given, rank 0, N=1 only;
  edgeconv_fwd_bwd_ms  the 4-block EdgeConv chain alone (fwd+bwd), and per block;
                       chain_fp32_exact / chain_fp32_split: the same chain in the
                       exact fp32 parity mode / the split-bf16 "fp32_split" mode;
  fp32_exact_mode / fp32_split_mode  the step in those two precisions;
  torch_eager_gpu      the reference op sequence in stock PyTorch-ROCm eager on
                       the same GPU, fp32 and under bf16 autocast.
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time
import types

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dgcnn.pytorch_amd"))

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 vector = f32 MFMA peak
PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)

METRIC = "point-clouds/sec + EdgeConv fwd+bwd ms at B=32 N=1024 k=20, 1/2/4/8 MI355X"
PRESETS = {"cfg2": (32, 1024, 20, 3), "cfg3": (32, 2048, 40, 3), "cfg5": (24, 4096, 20, 9)}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                   help="weak: --batch clouds per GPU; strong: --batch clouds in total, split over the GPUs")
    p.add_argument("--config", choices=sorted(PRESETS), default="cfg2",
                   help="BASELINE.json configs: cfg2 N1024 k20 B32 (headline), cfg3 N2048 k40 B32, "
                        "cfg5 N4096 k20 B24 on the 9-channel S3DIS block layout")
    p.add_argument("--batch", type=int, default=None, help="clouds per GPU (weak) or in total (strong)")
    p.add_argument("--points", type=int, default=None)
    p.add_argument("--k", type=int, default=None)
    p.add_argument("--emb", type=int, default=1024)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-eager-baseline", action="store_true")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--precision", choices=["bf16", "fp32", "fp32_split"], default="bf16",
                   help="GEMM operand precision (BASELINE cfg2 is bf16; fp32 is the exact parity mode; "
                        "fp32_split runs the fp32 GEMMs as 3-pass split bf16)")
    p.add_argument("--no-fp32-leg", action="store_true", help="skip the extra fp32 / fp32_split timings")
    p.add_argument("--no-edgeconv-leg", action="store_true", help="skip the EdgeConv-only fwd+bwd timing")
    p.add_argument("--no-posemb-leg", action="store_true",
                   help="skip the PositionEmbedding edge-MLP timing (partseg geometry)")
    p.add_argument("--no-graph", action="store_true",
                   help="N=1: time the eager-launched step instead of its HIP-graph replay")
    p.add_argument("--no-roofline-leg", action="store_true", help="skip the event-timed kNN region")
    p.add_argument("--no-attention-leg", action="store_true", help="skip the Net attention (f2) timing")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="collective backend for N>1 (nccl = RCCL on ROCm; gloo only to rehearse several ranks "
                        "on one GPU)")
    p.add_argument("--sgd", choices=["fused", "foreach", "dgx"], default="dgx",
                   help="SGD implementation: torch.optim.SGD fused / foreach, or dgx.optim.SGD (one HIP "
                        "launch); the same update")
    p.add_argument("--rccl-world1", action="store_true",
                   help="N=1: create a world-size-1 RCCL process group and take the N>1 step (flat-buffer "
                        "all-reduce after the graph-replayed fwd+bwd; with --sync-bn the BN-statistics "
                        "collectives too), so the multi-GPU code path runs on one GPU")
    p.add_argument("--sync-bn", action="store_true",
                   help="N>1: SyncBatchNorm (global-batch BN statistics, main_partseg_dist.py:189) instead of "
                        "per-replica BN (main_cls.py:62 DataParallel semantics)")
    a = p.parse_args(argv)
    preset = PRESETS[a.config]
    a.batch = a.batch or preset[0]
    a.points = a.points or preset[1]
    a.k = a.k or preset[2]
    a.in_dims = preset[3]
    return a


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args):
    """--gpus N without an outer launcher: run N ranks under torch.distributed.run
    as a child process (nothing in this process has touched the GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    return subprocess.call(cmd)


_GRADS = {}


def upstream_grad(shape, dev):
    """The loss head's gradient w.r.t. DGCNN's (B, emb, N) output: a fixed
    random tensor, made once outside every timed region. The reference DGCNN
    is an embedding net with no loss of its own (models/dgcnn.py:80-103); all
    legs (engine, eager PyTorch, CPU) back-propagate the same kind of dense
    upstream gradient."""
    import torch
    key = (tuple(shape), str(dev))
    if key not in _GRADS:
        g = torch.Generator().manual_seed(1234)
        _GRADS[key] = (torch.rand(tuple(shape), generator=g) - 0.5).to(dev)
    return _GRADS[key]


def reduce_elapsed(elapsed, world, dev):
    """The job's time for the timed region: the slowest rank's (max over ranks)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def replicas_in_sync(model, world, dev, distributed=None):
    """N > 1 (or a world-size-1 process group): every rank holds bitwise the
    same parameters after the timed steps (fp64 checksum of all parameters,
    min == max over ranks, two collectives). None without a process group."""
    import torch
    import torch.distributed as dist
    if not (distributed if distributed is not None else world > 1):
        return None
    with torch.no_grad():
        c = torch.stack([p.detach().double().sum() for p in model.parameters()]).sum().view(1)
    lo, hi = c.clone(), c.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool(lo.item() == hi.item())


def sync_all(world):
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def timed_region(step, steps, world):
    sync_all(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync_all(world)
    return time.perf_counter() - t0


def _ms(fn, reps, warm=2):
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def _ms_graph(fn, reps, warm=2):
    """ms per call of ``fn`` captured once as a HIP graph and replayed (the
    engine's GPU time, independent of the host's launch rate)."""
    import torch
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        fn()
    return _ms(graph.replay, reps, warm=1)


def edgeconv_legs(model, x, reps=10, chain_only=False):
    """The metric's second number: the 4-block EdgeConv chain alone, fwd+bwd
    (train-mode BN, grads w.r.t. W, gamma, beta), and each block on its own
    with synthetic features of its input width."""
    import torch
    from dgx.edgeconv import edgeconv_stack
    blocks = model.edge_blocks()
    g = {}

    def run(inp, blks):
        out = edgeconv_stack(inp, model.k, blks)
        key = tuple(out.shape)
        if key not in g:
            g[key] = torch.randn(key, device=out.device)
        out.backward(g[key])
    res = {"timing": "HIP-graph replay of each leg (fwd+bwd)",
           "chain": round(_ms_graph(lambda: run(x, blocks), reps), 3)}
    if chain_only:
        return res
    B, _, N = x.shape
    # block i runs on the features block i-1 produces from the same input (the
    # chain's own kNN graphs; random high-dimensional features would time the
    # hub-heavy graphs of Gaussian data instead)
    with torch.no_grad():
        feats = edgeconv_stack(x, model.k, blocks)
    off = 0
    for i, blk in enumerate(blocks):
        cin = blk[0].weight.shape[1] // 2
        if i == 0:
            xi = x
        else:
            xi = feats[:, off - cin:off].reshape(B, N, cin).permute(0, 2, 1).contiguous()
        off += blk[0].weight.shape[0]
        res[f"block{i + 1}"] = round(_ms_graph(lambda: run(xi, [blk]), reps), 3)
    return res


def eager_edgeconv_ms(x, k, autocast_dtype=None, reps=5):
    """The metric's EdgeConv number in stock PyTorch-ROCm eager: the reference's
    4 EdgeConv blocks (models/dgcnn.py:84-98: get_graph_feature -> Conv2d -> BN
    -> LeakyReLU -> max over k) fwd+bwd on this GPU, the same work
    edgeconv_fwd_bwd_ms["chain"] times for the engine."""
    return eager_reference_step_ms(x, k, None, autocast_dtype=autocast_dtype, reps=reps, chain_only=True)


def eager_reference_step_ms(x, k, emb, autocast_dtype=None, reps=5, chain_only=False):
    """The reference's DGCNN op sequence (models/dgcnn.py:6-103: matmul, sum,
    topk, index gather, repeat, cat, permute, conv, BN, LeakyReLU, max) in stock
    PyTorch-ROCm eager on this GPU: the single-GPU denominator of the >=10x
    goal; ``autocast_dtype`` runs it under torch.autocast (like for like with
    the engine's bf16 mode)."""
    import contextlib

    import torch
    import torch.nn as nn
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
    convs, c = [], x.shape[1]
    for w in widths:
        convs.append(nn.Sequential(nn.Conv2d(2 * c, w, 1, bias=False), nn.BatchNorm2d(w),
                                   nn.LeakyReLU(0.2, inplace=True)).to(dev))
        c = w
    c5 = None if chain_only else nn.Sequential(nn.Conv2d(512, emb, 1, bias=False), nn.BatchNorm2d(emb),
                                               nn.LeakyReLU(0.2, inplace=True)).to(dev)
    ctx = (torch.autocast("cuda", dtype=autocast_dtype) if autocast_dtype is not None
           else contextlib.nullcontext())

    def step():
        with ctx:
            h, feats = x, []
            for m in convs:
                h = m(gf(h)).max(dim=-1, keepdim=False)[0]
                feats.append(h)
            if chain_only:
                y = torch.cat(feats, dim=1)
            else:
                y = c5(torch.cat(feats, dim=1).unsqueeze(-1)).view(x.shape[0], -1, x.shape[2])
        y.backward(upstream_grad(y.shape, dev).to(y.dtype))
    return _ms(step, reps, warm=1)


def posemb_edge_leg(dev, B=32, N=2048, k=40, reps=5):
    """a6: PositionEmbedding's edge stage (reference models/layers.py:45-52:
    get_graph_feature -> conv1 -> conv2 -> max over k), fwd+bwd, at the partseg
    geometry (BASELINE cfg4 per GPU: B 32, N 2048, k 40): the engine's fused op
    (dgx.edgemlp) next to the reference's op sequence in PyTorch-ROCm eager."""
    import torch
    import torch.nn as nn
    from dgx.edgemlp import edge_mlp2
    torch.manual_seed(1)

    def blocks():
        return (nn.Sequential(nn.Conv2d(6, 64, 1, bias=False), nn.BatchNorm2d(64), nn.LeakyReLU(0.2)).to(dev),
                nn.Sequential(nn.Conv2d(64, 128, 1, bias=False), nn.BatchNorm2d(128), nn.LeakyReLU(0.2)).to(dev))
    x = (torch.rand(B, 3, N, device=dev) * 2 - 1).requires_grad_(True)
    g = torch.randn(B, 128, N, device=dev)
    c1, c2 = blocks()
    eager_blocks = blocks()

    def engine():
        edge_mlp2(x, k, c1, c2).backward(g)

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

    out = {"config": f"B={B} N={N} k={k}, conv 6->64->128, train-mode BN, fwd+bwd"}
    out["engine_ms"] = round(_ms_graph(engine, reps, warm=1), 3)
    out["engine_eager_launch_ms"] = round(_ms(engine, reps, warm=1), 3)
    try:
        out["torch_eager_gpu_ms"] = round(_ms(eager, reps, warm=1), 2)
        out["speedup"] = round(out["torch_eager_gpu_ms"] / out["engine_ms"], 2)
    except RuntimeError as e:
        out["torch_eager_gpu_ms"] = {"error": str(e)[:200]}
    return out


def attention_leg(dev, B=32, N=2048, E=512, H=4, p=0.5, reps=5):
    """f2: one attention of Net (reference models/model_partseg.py:167-171,
    187-191: nn.Transformer / nn.MultiheadAttention at the partseg geometry,
    BASELINE cfg4 per GPU: B 32, N 2048, emb 512, 4 heads, dropout 0.5), fp16
    operands as the reference's AMP run has them, fwd+bwd: the engine kernels
    (dgx.attention) next to torch's scaled_dot_product_attention."""
    import torch
    import torch.nn.functional as F
    from dgx.attention import attention
    g = torch.Generator(device=dev).manual_seed(0)
    D = E // H
    qkv = torch.randn((B, N, 3 * E), device=dev, generator=g).half()
    go = torch.randn((B, N, E), device=dev, generator=g).half()
    q, k, v = (qkv[..., i * E:(i + 1) * E].detach().clone().requires_grad_(True) for i in range(3))

    def engine():
        attention(q, k, v, H, p).backward(go)

    qh, kh, vh = (t.detach().reshape(B, N, H, D).transpose(1, 2).requires_grad_(True) for t in (q, k, v))
    goh = go.reshape(B, N, H, D).transpose(1, 2)

    def sdpa():
        F.scaled_dot_product_attention(qh, kh, vh, dropout_p=p).backward(goh)

    flops = 3.5 * 4.0 * B * H * N * N * D  # fwd 2 products + bwd 5 (FlashAttention accounting)
    out = {"config": f"B={B} N={N} E={E} heads={H} D={D} dropout={p}, fp16 operands, fwd+bwd"}
    out["engine_ms"] = round(_ms(engine, reps, warm=2), 3)
    out["engine_tflops"] = round(flops / (out["engine_ms"] * 1e-3) / 1e12, 1)
    try:
        out["torch_sdpa_ms"] = round(_ms(sdpa, reps, warm=2), 3)
        out["speedup"] = round(out["torch_sdpa_ms"] / out["engine_ms"], 2)
    except RuntimeError as e:
        out["torch_sdpa_ms"] = {"error": str(e)[:200]}
    return out


def _cgroup_cpus():
    """CPU quota of this process's cgroup (cgroup v2 cpu.max "quota period"),
    rounded up; None when unlimited or unreadable. On the GPU box the affinity
    set lists the whole machine while the quota is the box's share."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota == "max":
            return None
        return max(1, -(-int(quota) // int(period)))
    except (OSError, ValueError):
        return None


def cpu_baseline(args, clouds, sample_clouds=4, reps=None):
    """oracle/reference.py (torch-CPU restatement of the reference, pinned by
    tests/golden) timed on this job's host cores for DGCNN(emb) train fwd+bwd
    on the SAME batch the GPU step processes.

    The thread count is chosen by a sweep, not assumed: each candidate (powers
    of two up to the affinity set, plus the cgroup CPU quota) times one step on
    a ``sample_clouds``-cloud slice of the batch after a warm-up, stopping once
    two larger counts in a row are slower; the full batch is then timed at the
    best count (1 warm-up + ``reps``). More threads than the box's CPU share
    oversubscribe it (round 3: 256 threads took 28.6 s where 8 took 3.9 s)."""
    import torch
    from models.dgcnn import DGCNN
    sys.path.insert(0, REPO)
    from oracle import reference as R
    reps = max(3, args.cpu_reps if reps is None else reps)
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = _cgroup_cpus()
    cands = sorted({c for c in (1, 2, 4, 8, 16, 32, 64, 128, 256, avail, quota) if c and c <= avail})
    prev_threads = torch.get_num_threads()
    torch.manual_seed(0)
    model = DGCNN(types.SimpleNamespace(emb_dim=args.emb, k=args.k, in_dims=args.in_dims))
    params = {n: t.detach().clone() for n, t in model.state_dict().items()}
    for n, t in params.items():
        if t.is_floating_point() and "running" not in n:
            t.requires_grad_(True)
    x_all = torch.from_numpy(make_input(args, clouds, 0)).permute(0, 2, 1)

    def step(x):
        y, _ = R.dgcnn(x, args.k, params, training=True)
        y.backward(upstream_grad(y.shape, torch.device("cpu")))

    xs = x_all[:min(sample_clouds, clouds)]
    sweep, best, worse = {}, None, 0
    try:
        for c in cands:
            if c < 4 and avail >= 8:
                continue
            torch.set_num_threads(c)
            step(xs)
            t0 = time.perf_counter()
            step(xs)
            sweep[c] = round((time.perf_counter() - t0) * 1e3, 1)
            if best is None or sweep[c] < sweep[best]:
                best, worse = c, 0
            else:
                worse += 1
                if worse >= 2:
                    break
        torch.set_num_threads(best)
        step(x_all)
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            step(x_all)
            times.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev_threads)
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(clouds / med, 3), "unit": "clouds/s", "cores": best, "kind": "port",
            "host_cpus": os.cpu_count(), "affinity_cpus": avail, "cgroup_cpu_quota": quota,
            "thread_sweep_ms": {str(c): v for c, v in sweep.items()},
            "min_ms": round(times[0] * 1e3, 1), "median_ms": round(med * 1e3, 1), "reps": len(times),
            "sample": f"oracle/reference.py DGCNN(emb={args.emb}) train fwd+bwd on the full {clouds}-cloud batch "
                      f"({args.points} pts, k={args.k}); median of {len(times)} after 1 warm-up; torch CPU with "
                      f"{best} threads, chosen by thread_sweep_ms (one step of a {xs.shape[0]}-cloud slice per "
                      f"count; affinity set {avail} CPUs, cgroup quota {quota}, machine {os.cpu_count()})"}


def make_input(args, clouds, seed):
    from dgx import synth
    if args.in_dims == 9:
        return synth.s3dis_blocks(clouds, args.points, seed=2 + seed)
    return synth.cube_clouds(clouds, args.points, seed=seed)


def pmc_traffic(args, shapes, per_gpu):
    """HBM bytes per kNN selection launch from the committed rocprofv3 PMC
    summary of this config (profiles/*_pmc_<config>.json, newest round first),
    averaged over this step's launches. Returns (bytes or None, note): a file
    whose kernel names do not include every selection kernel this build
    launches for the step's layers is refused."""
    from dgx import _native as nat
    pb, pn, pk, _ = PRESETS[args.config]
    if (per_gpu, args.points, args.k) != (pb, pn, pk):
        # the committed counters are per launch of the preset's shapes; other
        # batch sizes launch other grids (and, for few clouds, other kernels)
        return None, f"no PMC profile for B={per_gpu} N={args.points} k={args.k} (committed: {args.config} preset)"
    names = [nat.lib().dgx_knn_kernel_name(c, args.k, args.points).decode() for c in shapes]
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"*_pmc_{args.config}.json")), reverse=True)
    if not files:
        return None, f"no profiles/*_pmc_{args.config}.json"
    with open(files[0]) as f:
        pmc = json.load(f)
    per = pmc.get("kernels", {})
    missing = sorted({n for n in names if n not in per})
    if missing:
        return None, f"{os.path.basename(files[0])} refused: no counters for {missing} (kernel names changed)"
    vals = [per[n]["hbm_bytes"] for n in names]
    return sum(vals) / len(vals), f"{os.path.basename(files[0])}: 2*FETCH_SIZE + WRITE_SIZE per launch, mean over {names}"


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))

    import torch
    import torch.distributed as dist
    from dgx import ops as dgx_ops
    from dgx import precision as dgx_prec
    from models.dgcnn import DGCNN

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if world > 1 and args.backend == "nccl" and ndev < world:
        raise SystemExit(f"{world} RCCL ranks need {world} GPUs, this node has {ndev}")
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    pg1 = world == 1 and args.rccl_world1
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    elif pg1:   # RCCL accepts a one-rank communicator: the N>1 path on one GPU
        from dgx import dist as dgx_dist
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=dev)
        if args.sync_bn:
            dgx_dist.sync_single_rank(True)   # torch would skip the sync at world 1; run the collective
    if args.scaling == "strong":
        if args.batch % world:
            raise SystemExit(f"--scaling strong: global batch {args.batch} does not split over {world} GPUs")
        per_gpu = args.batch // world
    else:
        per_gpu = args.batch
    total = per_gpu * world

    dgx_prec.set(args.precision)
    torch.manual_seed(0)
    model = DGCNN(types.SimpleNamespace(emb_dim=args.emb, k=args.k, in_dims=args.in_dims)).to(dev).train()
    net = model
    # N > 1: each rank's fwd + bwd is one HIP graph accumulating every
    # parameter gradient into ONE flat buffer, then ONE collective all-reduce
    # of it (sum / N: DDP's averaging) and the fused SGD step. With --sync-bn
    # over RCCL the BN-statistics all-reduces (no host synchronisation, dgx.dist)
    # are captured inside that graph; over gloo (host collectives, not
    # capturable) or with --no-graph the step runs eagerly under DDP
    distributed = world > 1 or pg1
    flat_dp = distributed and not args.no_graph and (not args.sync_bn or args.backend == "nccl")
    if distributed:
        if args.sync_bn:
            model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
        if flat_dp:
            with torch.no_grad():  # replicas start identical (what DDP's constructor does)
                for t in model.state_dict().values():
                    dist.broadcast(t, 0)
        else:
            net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = None
    if args.sgd == "dgx":   # the same update in one HIP launch (dgx/optim.py)
        from dgx.optim import SGD as DgxSGD
        opt = DgxSGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    elif args.sgd == "fused":
        try:  # one fused kernel for the whole parameter list (same math as the foreach form)
            opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, fused=True)
        except (RuntimeError, TypeError, ValueError):
            opt = None
    if opt is None:
        opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, foreach=True)
    pts = torch.from_numpy(make_input(args, per_gpu, seed=rank)).to(dev)
    x = pts.permute(0, 2, 1)  # (B,C,N) view, as main_cls.py:91 feeds the model

    gy = upstream_grad((per_gpu, args.emb, args.points), dev)

    if flat_dp:
        params = [p for p in model.parameters() if p.requires_grad]
        flat = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=dev)
        off = 0
        for p in params:  # every .grad is a view of the flat buffer: backward accumulates in place
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()

        def fwd_bwd():
            flat.zero_()
            net(x).backward(gy)

        def reduce_and_step():
            dist.all_reduce(flat)
            flat.mul_(1.0 / world)
            opt.step()

        def step():
            fwd_bwd()
            reduce_and_step()
    else:
        def step():
            opt.zero_grad(set_to_none=True)
            y = net(x)
            y.backward(gy)
            opt.step()

    for _ in range(args.warmup):
        step()
    # the same step launched eagerly (one C++ op + C++ autograd node issue the
    # ~60 launches of a step: dgx.host)
    elapsed_eager = reduce_elapsed(timed_region(step, args.steps, world), world, dev)
    launch = "eager"
    run = step
    elapsed_amp = None
    if world == 1 and not distributed:
        # the reference's own training configuration (main_partseg_dist.py:253): the
        # eager step under fp16 autocast with the engine's global mode at fp32 — the
        # GEMMs follow autocast to the split-bf16 path (16 significant bits per
        # operand, never narrower than fp16: dgx.precision.effective), issued
        # through the one-op C++ layer
        dgx_prec.set("fp32")

        def amp_step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.float16):
                y = net(x)
            y.backward(gy)
            opt.step()
        for _ in range(3):
            amp_step()
        elapsed_amp = timed_region(amp_step, args.steps, world)
        dgx_prec.set(args.precision)
    if world == 1 and not args.no_graph and not flat_dp:
        # one HIP graph per train step (fwd + bwd + SGD, the same kernels and
        # buffers as the eager step, captured once): replay issues the whole step
        # with one launch, independent of host speed. Grads are None when the
        # capture starts, so backward writes fresh gradient buffers (graph pool)
        # on every replay, as zero_grad(set_to_none=True) + backward does.
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(graph):
            net(x).backward(gy)
            opt.step()
        run = graph.replay
        for _ in range(2):
            run()
        launch = "hip_graph"
    elif flat_dp:
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                fwd_bwd()
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        # thread_local: the collective backend's watchdog thread may query events
        # while this thread captures (a global capture mode would reject that)
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            fwd_bwd()

        def run():
            graph.replay()
            reduce_and_step()
        for _ in range(2):
            run()
        launch = "hip_graph+allreduce" + ("(+syncbn collectives in graph)" if args.sync_bn else "")
    # headline: the timed region runs uninstrumented
    elapsed = reduce_elapsed(timed_region(run, args.steps, world), world, dev)
    result = {
        "metric": METRIC,
        "value": round(total * args.steps / elapsed, 2),
        "unit": "clouds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "launch": launch,
        "eager_launch_ms_per_step": round(elapsed_eager / args.steps * 1e3, 3),
        "autocast_eager_ms_per_step": (round(elapsed_amp / args.steps * 1e3, 3) if elapsed_amp is not None
                                       else None),
        "replicas_in_sync": replicas_in_sync(model, world, dev, distributed),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (splitmix64 uniform-cube clouds" + (", S3DIS 9-channel block layout" if args.in_dims == 9
                                                               else "") + ", random-init weights, fixed random "
                                                                          "upstream gradient)",
        "config": {"workload": f"DGCNN(emb={args.emb},k={args.k}) train step fwd+bwd+SGD, {args.config}",
                   "model": "DGCNN", "global_batch": total, "batch_per_gpu": per_gpu, "points": args.points,
                   "seq_len": args.points, "k": args.k, "emb_dim": args.emb, "in_channels": args.in_dims,
                   "parallelism": f"dp{world}" + ("+syncbn" if (args.sync_bn and distributed) else ""),
                   "backend": ("rccl" if args.backend == "nccl" or pg1 else "gloo") if distributed else "none",
                   "optimizer": {"dgx": "dgx.optim.SGD (one launch)", "fused": "torch.optim.SGD fused",
                                 "foreach": "torch.optim.SGD foreach"}[args.sgd]
                   + " lr 0.1 momentum 0.9 wd 1e-4"},
    }
    if not args.no_roofline_leg:
        # the same K steps again with HIP events around ONLY the kNN selection
        # launches (on their launch stream): 8 events per step
        timing = []
        dgx_ops.set_knn_timing(timing)
        elapsed_inst = reduce_elapsed(timed_region(step, args.steps, world), world, dev)
        dgx_ops.set_knn_timing(None)
        knn_ms = [e0.elapsed_time(e1) for (e0, e1, _, _) in timing]
        launches = max(1, len(knn_ms))
        avg_ms = sum(knn_ms) / launches
        avg_flops = sum(f for (_, _, f, _) in timing) / launches
        achieved = avg_flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
        per_layer = {}
        for (ms, (_, _, _, shape)) in zip(knn_ms, timing):
            per_layer.setdefault(f"C{shape[1]}", []).append(ms)
        per_layer = {c: round(sum(v) / len(v), 4) for c, v in per_layer.items()}
        shapes = [s[1] for (_, _, _, s) in timing[:4]]
        traffic, tnote = pmc_traffic(args, shapes, per_gpu)
        result["roofline"] = {
            "kernel": "knn_kernel (fused fp32 Gram on MFMA + top-k selection)", "bound": "mfma",
            "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": traffic, "traffic_source": tnote,
            "avg_launch_ms": round(avg_ms, 4), "algorithmic_flops_per_launch": avg_flops,
            "launches_timed": len(knn_ms), "knn_ms_by_layer": per_layer,
            "timed_region": "second K-step region, events around the kNN selection launches only "
                            "(ms_per_step %.3f)" % (elapsed_inst / args.steps * 1e3)}
    if not args.no_fp32_leg:
        # the same model in the exact fp32 parity mode and in the split-bf16
        # "fp32_split" mode (NOT exact fp32: ~2^-16 per product), eager launch
        n32 = max(2, args.steps // 2)
        for mode in ("fp32", "fp32_split"):
            if mode == args.precision:
                continue
            dgx_prec.set(mode)
            for _ in range(3):  # warm-up
                step()
            el32 = reduce_elapsed(timed_region(step, n32, world), world, dev)
            result[{"fp32": "fp32_exact_mode", "fp32_split": "fp32_split_mode"}[mode]] = {
                "ms_per_step": round(el32 / n32 * 1e3, 3), "value": round(total * n32 / el32, 2),
                "launch": "eager"}
        dgx_prec.set(args.precision)
    if rank == 0 and world == 1:
        if not args.no_edgeconv_leg:
            legs = edgeconv_legs(model, x)
            for mode in ("fp32", "fp32_split"):   # the fp32 modes' chains beside stock fp32 eager
                dgx_prec.set(mode)
                legs[f"chain_{'fp32_exact' if mode == 'fp32' else mode}"] = edgeconv_legs(
                    model, x, chain_only=True)["chain"]
            dgx_prec.set(args.precision)
            if not args.no_eager_baseline:
                # the same 4-block chain in stock PyTorch-ROCm eager (the metric's EdgeConv ratio)
                for name, dt in (("fp32", None), ("bf16_autocast", torch.bfloat16)):
                    try:
                        legs[f"torch_eager_{name}"] = round(eager_edgeconv_ms(x, args.k, autocast_dtype=dt), 3)
                    except RuntimeError as e:
                        legs[f"torch_eager_{name}"] = {"error": str(e)[:200]}
                    torch.cuda.empty_cache()
                ref = legs.get(f"torch_eager_{'bf16_autocast' if args.precision == 'bf16' else 'fp32'}")
                if isinstance(ref, float):
                    legs["engine_speedup_vs_eager"] = round(ref / legs["chain"], 2)
                if isinstance(legs.get("torch_eager_fp32"), float):
                    # exact fp32 vs torch fp32: the same arithmetic class
                    legs["fp32_exact_speedup_vs_eager_fp32"] = round(legs["torch_eager_fp32"] /
                                                                     legs["chain_fp32_exact"], 2)
                    # split-bf16 products (~2^-16) vs torch's exact fp32: NOT the same precision
                    legs["fp32_split_speedup_vs_eager_fp32"] = round(legs["torch_eager_fp32"] /
                                                                     legs["chain_fp32_split"], 2)
            result["edgeconv_fwd_bwd_ms"] = legs
        if not args.no_posemb_leg:
            result["posemb_edge_mlp"] = posemb_edge_leg(dev)
        if not args.no_attention_leg:
            result["net_attention"] = attention_leg(dev)
        if not args.no_eager_baseline:
            eager = {}
            ours32 = result["ms_per_step"] if args.precision == "fp32" else result.get("fp32_exact_mode", {}).get(
                "ms_per_step")
            ours16 = result["ms_per_step"] if args.precision == "bf16" else None
            for name, dt, ours in (("fp32", None, ours32), ("bf16_autocast", torch.bfloat16, ours16)):
                try:
                    ms = eager_reference_step_ms(x, args.k, args.emb, autocast_dtype=dt)
                    eager[name] = {"ms_per_step": round(ms, 2), "clouds_per_s": round(per_gpu / ms * 1e3, 2)}
                    if ours:
                        eager[name]["engine_speedup"] = round(ms / ours, 2)
                except RuntimeError as e:  # e.g. out of memory: report, don't hide
                    eager[name] = {"error": str(e)[:200]}
                torch.cuda.empty_cache()
            eager["note"] = ("engine_speedup: fp32 eager vs the engine's exact fp32 mode (fp32_exact_mode, eager "
                             "launch), bf16-autocast eager vs the engine's bf16 mode (the headline step)")
            result["torch_eager_gpu"] = eager
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args, per_gpu)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
