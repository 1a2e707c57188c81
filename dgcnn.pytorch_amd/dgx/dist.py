"""Cross-rank BatchNorm statistics for the engine's fused BN (SyncBatchNorm).

Reference: main_partseg_dist.py:189 wraps the model with
``nn.SyncBatchNorm.convert_sync_batchnorm`` before DDP, so every BN layer of
the EdgeConv chain and conv5 normalises with the statistics of the GLOBAL batch
(torch/nn/modules/_functions.py: forward all-gathers per-rank mean/invstd/count,
backward all-reduces sum(dy) and sum(dy * xmu)).

The engine keeps those exact semantics with one collective per BN layer and
direction: the kernels already produce per-block partial sums, the host sums
them in fp64 to one (2, C) vector, and ``allreduce_sums`` adds the vectors of
all ranks (plus the element count) in a single fp64 all-reduce over RCCL (or
gloo). The global sums stay fp64 into the finalize kernel
(dgx_bn_finalize_f64), so var = E[y^2] - E[y]^2 sees no fp32 round trip.
Parameter gradients stay rank-local (DDP averages them), exactly as
SyncBatchNorm does.
"""
import torch
import torch.distributed as dist
import torch.nn as nn

# Smallest process-group size at which a SyncBatchNorm synchronises. torch's
# SyncBatchNorm skips the collective on a single rank (need_sync = world > 1);
# the engine does the same by default. ``sync_single_rank(True)`` lowers it to
# 1 so the collective path (fp64 sums all-reduced over RCCL, inside a HIP graph
# or from the C++ op) runs on a one-GPU box with a world-size-1 RCCL group
# (tests/test_rccl_gpu.py, bench.py --rccl-world1).
_MIN_WORLD = 2


def sync_single_rank(on):
    global _MIN_WORLD
    _MIN_WORLD = 1 if on else 2


def sync_group(bn):
    """(True, group) when ``bn`` is a SyncBatchNorm that must synchronise now
    (SyncBatchNorm.forward: batch statistics in training mode, world > 1)."""
    if not (bn.training and isinstance(bn, nn.SyncBatchNorm)):
        return False, None
    if not (dist.is_available() and dist.is_initialized()):
        return False, None
    group = bn.process_group if bn.process_group is not None else dist.group.WORLD
    if dist.get_world_size(group) < _MIN_WORLD:
        return False, None
    return True, group


def allreduce_sums(partials, count, group):
    """partials: (rows, 2, C) fp32 per-block column sums; count: local element
    count. Returns the (2C + 1) fp64 buffer [global sums (2, C) | global count]
    after ONE all-reduce. The count stays on the device: the fp64 finalize
    kernels read it there (count argument -1), so no host synchronisation sits
    on the SyncBatchNorm critical path and the step stays graph-capturable."""
    C = partials.shape[-1]
    buf = torch.empty(2 * C + 1, dtype=torch.float64, device=partials.device)
    torch.sum(partials.double(), dim=0, out=buf[:2 * C].view(2, C))
    buf[2 * C:].fill_(float(count))
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf
