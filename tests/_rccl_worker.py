"""Worker for tests/test_rccl_gpu.py: the engine's multi-GPU step on ONE GPU
over a world-size-1 RCCL process group (torch.distributed "nccl", which is
RCCL on ROCm; reference main_partseg_dist.py:486 init_process_group('nccl'),
:189-196 SyncBatchNorm + DDP).

RCCL accepts a one-rank communicator, so every code path the driver's 8-GPU
run takes first executes here on hardware:
  flat     bench.py's N>1 step: fwd+bwd captured as one HIP graph whose
           backward accumulates every gradient into ONE flat buffer, then one
           RCCL all-reduce of it, the 1/world scale and the one-launch SGD;
  ddp      torch DDP (bucketed RCCL all-reduce overlapped with backward);
  sync     SyncBatchNorm forced to synchronise at world 1
           (dgx.dist.sync_single_rank): the fp64 BN sums all-reduced from the
           C++ op (_c10d_functional::all_reduce_), eagerly ...
  syncg    ... and captured inside the fwd+bwd HIP graph with the flat buffer.
Each runs STEPS SGD steps from the same initial weights on the same batch; the
worker writes every run's last output, gradients, parameters and BatchNorm
buffers to <out>/rccl1.pt for the test to compare with the plain
single-process step (no process group)."""
import os
import socket
import sys
import types

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]

STEPS = 3
ARGS = dict(emb_dim=256, k=20)
B, N = 8, 1024


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    out_dir, precision = sys.argv[1], sys.argv[2]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    from dgx import dist as dgx_dist
    from dgx import precision as prec
    from dgx import synth
    from dgx.optim import SGD
    from models.dgcnn import DGCNN
    prec.set(precision)
    x = torch.from_numpy(synth.cube_clouds(B, N, 7)).to(dev).permute(0, 2, 1)
    gy = torch.from_numpy(synth.uniform(8, (B, ARGS["emb_dim"], N)) - 0.5).to(dev)

    def make(sync):
        torch.manual_seed(0)
        m = DGCNN(types.SimpleNamespace(**ARGS))
        if sync:
            m = torch.nn.SyncBatchNorm.convert_sync_batchnorm(m)
        return m.to(dev).train()

    def record(m, y):
        torch.cuda.synchronize()
        return {"y": y.detach().float().cpu().clone(),
                "grads": {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()},
                "params": {n: p.detach().cpu().clone() for n, p in m.named_parameters()},
                "buffers": {n: b.detach().cpu().clone() for n, b in m.named_buffers()}}

    def eager(m, net):
        opt = SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        for _ in range(STEPS):
            opt.zero_grad(set_to_none=True)
            y = net(x)
            y.backward(gy)
            opt.step()
        return record(m, y)

    def flat_graph(m):
        """bench.py's flat_dp branch: the graph is captured after two warm-up
        steps, so its first replay is step 3."""
        params = [p for p in m.parameters() if p.requires_grad]
        flat = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=dev)
        off = 0
        for p in params:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        opt = SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        ys = []

        def fwd_bwd():
            flat.zero_()
            y = m(x)
            y.backward(gy)
            return y

        def reduce_and_step():
            dist.all_reduce(flat)
            flat.mul_(1.0 / dist.get_world_size())
            opt.step()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(STEPS - 1):
                ys.append(fwd_bwd())
                reduce_and_step()
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        # the capture does not run the kernels: the parameters stay at step STEPS-1
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            y_static = fwd_bwd()
        graph.replay()
        reduce_and_step()
        return record(m, y_static)

    res = {"plain": None}
    m = make(False)
    res["flat"] = flat_graph(m)
    m = make(False)
    res["ddp"] = eager(m, torch.nn.parallel.DistributedDataParallel(m, device_ids=[0]))
    dgx_dist.sync_single_rank(True)
    try:
        m = make(True)
        res["sync"] = eager(m, m)
        m = make(True)
        res["syncg"] = flat_graph(m)
    finally:
        dgx_dist.sync_single_rank(False)
    dist.barrier()
    dist.destroy_process_group()
    # the reference point: the same steps with no process group at all
    m = make(False)
    res["plain"] = eager(m, m)
    torch.save(res, os.path.join(out_dir, "rccl1.pt"))


if __name__ == "__main__":
    main()
