"""BatchNorm bookkeeping shared by the engine's fused layers.

The reference's EdgeConv blocks, conv5 and PositionEmbedding convs are
``nn.BatchNorm2d`` modules (models/dgcnn.py:54-78, models/layers.py:14-20).
The engine folds their arithmetic into its kernels but takes every decision
the way ``nn.BatchNorm``'s own forward takes it, per BN module:

* batch statistics when ``bn.training`` or the module tracks no running
  statistics; running statistics otherwise (e.g. ``model.train()`` with the BN
  layers frozen in ``eval()``);
* running statistics updated only when ``bn.training`` and
  ``bn.track_running_stats``, with momentum or the cumulative average;
* SyncBatchNorm (main_partseg_dist.py:189) synchronises only in training mode.

Backward: train mode gives BN's full input gradient, dy = a*dz + c0 + c1*y
per element (c0, c1 from the fp64 finalize); eval mode is the fixed affine,
dy = a*dz (c0 = c1 = 0), with dgamma/dbeta over the running-statistics yhat.
"""
from collections import namedtuple

import torch

from . import _native as nat
from . import dist as dist_

# per-channel fp32 tensors (Co,) + the SyncBatchNorm process group (or None)
# + whether the running statistics normalised this forward
Stats = namedtuple("Stats", "scale shift mean invstd group eval")


def mode(bn):
    """(use batch statistics, update running statistics) — nn.BatchNorm's rule."""
    use_batch = bn.training or (bn.running_mean is None and bn.running_var is None)
    update = bool(bn.training and bn.track_running_stats and bn.running_mean is not None)
    return use_batch, update


def op_args(bn):
    """One BN layer's arguments for the C++ schedule (libdgx_torch.so,
    dgx_host::chain_* / pointconv_* / dgcnn): ([running_mean, running_var,
    num_batches_tracked, and the three update targets of a functional caller
    (``bn.stats_out``) or None for in place], [momentum (-1 = None), eps],
    [training, track_running_stats], SyncBatchNorm process-group name or "").
    The C++ side takes every decision of ``mode`` / ``batch_stats`` /
    ``running_stats`` / ``backward_consts`` from these, as nn.BatchNorm does."""
    out = getattr(bn, "stats_out", None)
    rm_o, rv_o, nb_o = out if out is not None else (None, None, None)
    sync, group = dist_.sync_group(bn)
    return ([bn.running_mean, bn.running_var, bn.num_batches_tracked, rm_o, rv_o, nb_o],
            [-1.0 if bn.momentum is None else float(bn.momentum), float(bn.eps)],
            [int(bool(bn.training)), int(bool(bn.track_running_stats))],
            group.group_name if sync else "")


def _factor(bn):
    """(exponential-average factor nn.BatchNorm uses this step, num_batches_tracked
    tensor for the finalize kernel to increment or None). With a momentum the
    counter is bumped on device by the finalize kernel (no extra launch); the
    cumulative-average form (momentum None) needs the count on the host."""
    if bn.momentum is None:
        if bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
            return 1.0 / float(bn.num_batches_tracked.item()), None
        return 0.0, None
    return float(bn.momentum), bn.num_batches_tracked


def _vec(co, dev):
    return torch.empty(co, dtype=torch.float32, device=dev)


def _compact(partials, rows, co, stream):
    """Pre-reduce a tall (rows, 2, co) partial array (the per-tile partials of
    the edge-MLP epilogues reach E/128 rows) to about 128 rows with the
    fixed-order slab sum, so the finalize kernels read few rows (deterministic:
    the grouping depends only on rows)."""
    if rows <= 1024:
        return partials, rows
    R = 128
    S = rows // R
    left = rows - S * R
    out = torch.empty((R + left, 2, co), dtype=torch.float32, device=partials.device)
    nat.check(nat.lib().dgx_slab_reduce_f32(nat.f32(partials), S, R, 2 * co, R, nat.f32(out), 2 * co, stream),
              "bn partial reduce")
    if left:
        out[R:].copy_(partials.view(-1, 2, co)[S * R:rows])
    return out, R + left


def _update_targets(bn):
    """Where the updated running statistics go: ``bn.stats_out`` = (mean, var,
    batch counter) tensors of a functional caller (dgx.library: the module
    buffers are read, the new values written there — no private copy first),
    else the module's own buffers, in place."""
    out = getattr(bn, "stats_out", None)
    if out is None:
        return bn.running_mean, bn.running_var, bn.num_batches_tracked
    return out


def batch_stats(partials, rows, count, bn, gamma, beta, stream):
    """Finalize batch statistics from per-block (sum y, sum y^2) partials
    (rows, 2, Co) over ``count`` elements; updates running statistics as
    nn.BatchNorm would (into ``bn.stats_out`` when the caller gives one)."""
    L = nat.lib()
    dev = partials.device
    co = gamma.shape[0]
    scale, shift, mean, invstd = _vec(co, dev), _vec(co, dev), _vec(co, dev), _vec(co, dev)
    _, update = mode(bn)
    rm_new, rv_new, nbt_new = _update_targets(bn)
    if update and getattr(bn, "stats_out", None) is not None and bn.momentum is None:
        # cumulative average (momentum=None): the finalize reads the counter and
        # uses 1 / (count + 1) on the device (factor -1), writing count + 1 to the
        # op's own output — no host read, so the op stays graph-capturable
        if bn.num_batches_tracked is not None:
            factor, nbt = -1.0, bn.num_batches_tracked
        else:
            factor, nbt = 0.0, None
    else:
        factor, nbt = _factor(bn) if update else (0.0, None)
    rm = nat.f32(bn.running_mean) if update else None
    rv = nat.f32(bn.running_var) if update else None
    outs = (nat.f32(rm_new) if update else None, nat.f32(rv_new) if update else None,
            nat.ptr(nbt_new, nat.I64) if nbt is not None else None)
    sync, group = dist_.sync_group(bn)
    partials, rows = _compact(partials, rows, co, stream)
    if sync:  # SyncBatchNorm: statistics of the global batch, one fp64 all-reduce
        sums = dist_.allreduce_sums(partials, count, group)   # (2C + 1) fp64: sums | global count
        nat.check(L.dgx_bn_finalize_out_f64(nat.ptr(sums, nat.F64), 1, co, -1.0, nat.f32(gamma), nat.f32(beta), rm,
                                            rv, factor, float(bn.eps), nat.f32(scale), nat.f32(shift), nat.f32(mean),
                                            nat.f32(invstd), nat.ptr(nbt, nat.I64), *outs, stream), "bn finalize")
    else:
        nat.check(L.dgx_bn_finalize_out_f32(nat.f32(partials), rows, co, float(count), nat.f32(gamma), nat.f32(beta),
                                            rm, rv, factor, float(bn.eps), nat.f32(scale), nat.f32(shift),
                                            nat.f32(mean), nat.f32(invstd), nat.ptr(nbt, nat.I64), *outs, stream),
                  "bn finalize")
    return Stats(scale, shift, mean, invstd, group if sync else None, False)


def running_stats(bn, gamma, beta, stream):
    """Eval-mode affine (scale, shift) from the running statistics, and the
    running mean / invstd that define yhat for dgamma if the output is
    differentiated."""
    L = nat.lib()
    dev = gamma.device
    co = gamma.shape[0]
    scale, shift = _vec(co, dev), _vec(co, dev)
    nat.check(L.dgx_bn_eval_affine_f32(co, nat.f32(gamma), nat.f32(beta), nat.f32(bn.running_mean),
                                       nat.f32(bn.running_var), float(bn.eps), nat.f32(scale), nat.f32(shift), stream),
              "bn eval affine")
    mean = bn.running_mean.detach().clone()
    invstd = torch.rsqrt(bn.running_var.detach() + bn.eps)
    return Stats(scale, shift, mean, invstd, None, True)


def backward_consts(partials, rows, count, st, stream):
    """(dgamma, dbeta, c0, c1) from per-block (sum g, sum g*yhat) partials, where
    g is the gradient w.r.t. the BN output at every element: BN's train-mode
    input gradient a*g + c0 + c1*y, or the eval-mode affine (c0 = c1 = 0)."""
    L = nat.lib()
    dev = partials.device
    co = st.scale.shape[0]
    dgamma, dbeta, c0, c1 = _vec(co, dev), _vec(co, dev), _vec(co, dev), _vec(co, dev)
    args = (nat.f32(st.scale), nat.f32(st.mean), nat.f32(st.invstd))
    partials, rows = _compact(partials, rows, co, stream)
    if st.group is None:
        nat.check(L.dgx_bn_bwd_finalize_f32(nat.f32(partials), rows, co, float(count), *args, nat.f32(dgamma),
                                            nat.f32(dbeta), nat.f32(c0), nat.f32(c1), 0, stream), "bn bwd finalize")
        if st.eval:
            c0.zero_()
            c1.zero_()
    else:  # SyncBatchNorm: input gradient from global sums, gamma/beta grads rank-local
        sums = dist_.allreduce_sums(partials, count, st.group)
        nat.check(L.dgx_bn_bwd_finalize_f64(nat.ptr(sums, nat.F64), 1, co, -1.0, *args, None, None, nat.f32(c0),
                                            nat.f32(c1), 0, stream), "bn bwd finalize")
        loc = partials.double().sum(0)
        dbeta.copy_(loc[0])
        dgamma.copy_(loc[1])
    return dgamma, dbeta, c0, c1
