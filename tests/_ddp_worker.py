"""Worker for tests/test_ddp_gpu.py: one rank of a world-size-2 DDP run of the
engine's DGCNN on cuda:0 (gloo backend, both ranks share the GPU). Writes its
outputs and (DDP-averaged) gradients to <out>/rank<r>.pt."""
import os
import sys
import types

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    out_dir, mode, precision = sys.argv[1], sys.argv[2], sys.argv[3]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dgx import precision as prec
    from dgx import synth
    from models.dgcnn import DGCNN
    from models.layers import PositionEmbedding
    prec.set(precision)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    posemb = mode.startswith("posemb")
    if mode == "net_syncbn_amp":
        return net_syncbn_amp(rank, world, out_dir, dev)
    if mode == "dgcnn_syncbn_amp":
        return dgcnn_syncbn_amp(rank, world, out_dir, dev)
    if posemb:  # PositionEmbedding (a6) as main_partseg_dist.py converts Net's modules
        model = PositionEmbedding(types.SimpleNamespace(k=10))
        with torch.no_grad():
            model.transform.weight.normal_(0, 0.05)
    else:
        model = DGCNN(types.SimpleNamespace(emb_dim=64, k=10))
    if mode.endswith("syncbn"):
        model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
    model = model.to(dev).train()
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0])
    B = 2
    pts = synth.cube_clouds(B * world, 256, 5)[rank * B:(rank + 1) * B]
    x = torch.from_numpy(pts).to(dev).permute(0, 2, 1)
    y = ddp(x)
    co = 3 if posemb else 64
    g = torch.from_numpy(synth.uniform(6, (B * world, co, 256)) - 0.5)[rank * B:(rank + 1) * B].to(dev)
    (y * g).sum().backward()
    torch.cuda.synchronize()
    res = {"y": y.detach().cpu(),
           "grads": {n: p.grad.detach().cpu() for n, p in model.named_parameters() if p.grad is not None},
           "running": {n: b.detach().cpu() for n, b in model.named_buffers()}}
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


AMP_ARGS = dict(emb_dim=512, k=40)   # DGCNN as Net's emb_nn builds it at cfg4 (main_partseg_dist.py:534)
AMP_B, AMP_N = 2, 2048


def amp_inputs(world):
    from dgx import synth
    pts = synth.cube_clouds(AMP_B * world, AMP_N, 41)
    g = torch.from_numpy(synth.uniform(42, (AMP_B * world, AMP_ARGS["emb_dim"], AMP_N)) - 0.5).float()
    return pts, g


def dgcnn_syncbn_amp(rank, world, out_dir, dev):
    """DGCNN (the engine) converted with SyncBatchNorm under DDP, forward under
    fp16 autocast (main_partseg_dist.py:189-196, 253): bf16 GEMMs, BatchNorm
    statistics of the global batch all-reduced from the C++ op."""
    from models.dgcnn import DGCNN
    torch.manual_seed(0)
    model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(DGCNN(types.SimpleNamespace(**AMP_ARGS))).to(dev).train()
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0])
    pts, g = amp_inputs(world)
    sl = slice(rank * AMP_B, (rank + 1) * AMP_B)
    x = torch.from_numpy(pts[sl]).to(dev).permute(0, 2, 1)
    with torch.autocast("cuda", dtype=torch.float16):
        y = ddp(x)
    (y.float() * g[sl].to(dev)).sum().backward()
    torch.cuda.synchronize()
    res = {"y": y.detach().float().cpu(),
           "grads": {n: p.grad.detach().float().cpu() for n, p in model.named_parameters()},
           "running": {n: b.detach().cpu() for n, b in model.named_buffers()}}
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


NET_ARGS = dict(k=40, emb_dim=512, n_heads=4, n_blocks=1, ff_dims=512, dropout=0.0, nclasses=50)
NET_B, NET_N = 2, 2048   # clouds per rank, points (BASELINE cfg4 geometry, batch reduced)


def net_inputs(world):
    """Clouds arranged so every rank's first cloud is the global batch's first:
    compute_hog_1x1 gathers neighbourhoods with local ids from x.view(B*N, 3)
    (reference model_partseg.py:26-30), so a cloud's HOG depends
    on its batch's cloud 0 — a rank's outputs equal the full batch's only if
    those coincide."""
    import numpy as np
    from dgx import synth
    assert NET_B == 2 and world == 2
    c = synth.cube_clouds(3, NET_N, 31)
    pts = np.ascontiguousarray(np.stack([c[0], c[1], c[0], c[2]]))
    lbl = torch.nn.functional.one_hot(torch.arange(NET_B * world) % 16, 16).float()
    g = torch.from_numpy(synth.uniform(32, (NET_B * world, NET_N, NET_ARGS["nclasses"])) - 0.5).float()
    return pts, lbl, g


def net_syncbn_amp(rank, world, out_dir, dev):
    """Net as main_partseg_dist.py:189-196, 253-260 trains it: converted with
    SyncBatchNorm, wrapped in DDP, forward under fp16 autocast, backward of the
    unscaled loss (a fixed 2^10 scale overflows the stock fp16 layers'
    gradients here — GradScaler would skip that step and back off; the
    GradScaler loop itself is tests/test_amp_bn_gpu.py::
    test_net_autocast_grad_scaler). The engine's DGCNN (one C++ op)
    all-reduces its BN statistics over the module's process group from C++."""
    from models.model_partseg import Net
    # both ranks share cuda:0; compute_hog_1x1 moves its histograms to device
    # LOCAL_RANK as the reference does (model_partseg.py:66-73)
    os.environ["LOCAL_RANK"] = "0"
    torch.manual_seed(0)
    model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(Net(types.SimpleNamespace(**NET_ARGS))).to(dev).train()
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0])
    pts, lbl, g = net_inputs(world)
    sl = slice(rank * NET_B, (rank + 1) * NET_B)
    x = torch.from_numpy(pts[sl]).to(dev).permute(0, 2, 1).contiguous()
    scale = 1.0
    with torch.autocast("cuda", dtype=torch.float16):
        y = ddp(x, lbl[sl].to(dev))
    ((y.float() * g[sl].to(dev).permute(0, 2, 1)).sum() * scale).backward()
    torch.cuda.synchronize()
    res = {"y": y.detach().float().cpu(),
           "grads": {n: (p.grad.detach().float() / scale).cpu() for n, p in model.named_parameters()
                     if p.grad is not None},
           "running": {n: b.detach().cpu() for n, b in model.named_buffers()}}
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
