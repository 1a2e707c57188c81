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


if __name__ == "__main__":
    main()
