"""world_size-2 gloo tests on CPU (no GPU): the SyncBatchNorm statistics
all-reduce of dgx.dist (one collective per BN layer: column sums + count) and
the bench's max-over-ranks timing reduction."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _worker(rank, world, port, q):
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dgx import dist as D
        import bench
        # per-block partials (rows, 2, C): summed in fp64 locally, then across ranks
        part = torch.arange(12, dtype=torch.float32).view(2, 2, 3) * (rank + 1)
        buf = D.allreduce_sums(part, 10 + rank, dist.group.WORLD)
        # one fp64 buffer [sums (2, C) | count]: the count stays with the sums (read on the device)
        assert buf.dtype == torch.float64 and buf.is_contiguous() and buf.shape == (7,)
        tot, cnt = buf[:6].view(2, 3), float(buf[6])
        bn = torch.nn.SyncBatchNorm(3)
        on, grp = D.sync_group(bn.train())
        off, _ = D.sync_group(bn.eval())
        plain, _ = D.sync_group(torch.nn.BatchNorm2d(3))
        t = bench.reduce_elapsed(0.5 + rank, world, torch.device("cpu"))
        q.put((rank, tot.tolist(), cnt, on, off, plain, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_syncbn_stats_allreduce_and_bench_timing_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = (torch.arange(12, dtype=torch.float64).view(2, 2, 3).sum(0) * 3).tolist()
    for rank, tot, cnt, on, off, plain, t in res:
        assert tot == exp and cnt == 21.0
        assert on and not off and not plain
        assert t == 1.5  # every rank reports the slowest rank's time


def test_sync_group_needs_initialised_world():
    sys.path[:0] = [PKG]
    from dgx import dist as D
    assert D.sync_group(torch.nn.SyncBatchNorm(4)) == (False, None)
