"""torch.library op layer of the engine (SURVEY §8(b) "Torch op layer").

The reference's hot path is plain Python over ATen ops (models/dgcnn.py:6,
15, 47-103). The engine's HIP work is exposed here as ``torch.ops.dgx.*``
custom ops with device ("cuda" = ROCm) kernels, fake (meta) kernels for
tracing, autocast rules and autograd formulas, so ``torch.compile`` /
``torch.export`` / FX see each op as one node instead of an opaque ctypes call
(the compiled graph has no break at the engine):

  dgx::knn(x, k) -> int64 (B, N, k)                     dgcnn.py:6-12
  dgx::graph_feature(x, k, mode) -> (edge tensor, idx)  dgcnn.py:15-44
      (+ dgx::graph_feature_backward)
  dgx::weight_prep(weights, ...) -> bf16 operand buffer  (bf16 mode)
  dgx::edgeconv_chain(x, k, conv/BN tensors, ...) -> (concat buffer, its
      bf16 twin, updated running statistics, saved state)  dgcnn.py:84-100
      (+ dgx::edgeconv_chain_backward)
  dgx::pointconv(X, X16, B, N, conv/BN tensors, ...) -> (out, updated
      running statistics, saved state)                   dgcnn.py:100-102
      (+ dgx::pointconv_backward)

The ops are functional: BatchNorm running statistics come back as outputs (the
finalize kernels read the module buffers and write the new values straight
into the outputs: no private copy first) and the caller copies them into the
module buffers (what a compiled graph does with a buffer mutation anyway;
torch does not allow an autograd formula on an op that mutates its inputs).
The chain and conv5 ops run the C++ schedule (libdgx_torch.so,
dgx_host::chain_* / pointconv_*) that the eager DGCNN op and the engine's
autograd Functions run too, so eager results are identical either way;
``models.dgcnn.DGCNN`` takes this path while torch.compile traces it, unless a
BatchNorm is a SyncBatchNorm (process groups cannot cross the op boundary).
"""
from typing import Optional

import torch
from torch import Tensor

from . import bn as bn_
from . import cpu
from . import edgeconv as E
from . import gemm as G
from . import ops
from . import precision as prec

ENABLED = True
_F32, _BF16, _I32 = torch.float32, torch.bfloat16, torch.int32


def _empty(dev, dtype=_F32):
    return torch.empty(0, dtype=dtype, device=dev)


class _Rec:
    """The autograd-context surface the engine's Functions use, recorded so a
    custom op can run a Function's forward / backward body."""

    def __init__(self):
        self.saved_tensors = ()
        self.needs_input_grad = (True,) * 64

    def save_for_backward(self, *t):
        self.saved_tensors = t

    def mark_non_differentiable(self, *_):
        pass

    def set_materialize_grads(self, _):
        pass


class _BNSpec:
    """The nn.BatchNorm fields dgx.bn reads, rebuilt from tensors that crossed
    the op boundary (the running statistics are read from the inputs and the
    updates written to the op's outputs, ``out``)."""

    def __init__(self, training, track, rm, rv, nbt, momentum, eps, out=None):
        self.training = bool(training)
        self.track_running_stats = bool(track)
        self.running_mean = rm if rm.numel() else None
        self.running_var = rv if rv.numel() else None
        self.num_batches_tracked = nbt if nbt.numel() else None
        self.momentum = None if momentum < 0 else float(momentum)
        self.eps = float(eps)
        # (mean, var, counter) outputs the finalize writes the updated statistics
        # to (dgx.bn._update_targets); the inputs are only read
        self.stats_out = out


def _use_batch(training, rm):
    return bool(training) or rm.numel() == 0


def _copy_many(dsts, srcs):
    """dst_i <- src_i for many small tensors in one multi-tensor launch per
    dtype (the BN running statistics cross the functional op boundary as
    private copies: 2 launches per step instead of one per tensor)."""
    groups = {}
    for d, s in zip(dsts, srcs):
        if d.numel():
            groups.setdefault(d.dtype, ([], []))
            groups[d.dtype][0].append(d)
            groups[d.dtype][1].append(s)
    for ds, ss in groups.values():
        torch._foreach_copy_(ds, ss)


def _stat_outputs(training, track, rms, rvs, nbts):
    """The ops' running-statistics outputs (distinct storages: op outputs may
    not alias inputs). A layer that updates them (training and tracking) gets
    uninitialised tensors the finalize kernel fills from the inputs; the others
    get copies of the inputs, all in one multi-tensor launch per dtype (none
    in a training step)."""
    outs, dsts, srcs = [], [], []
    for tr, tk, rm, rv, nb in zip(training, track, rms, rvs, nbts):
        o = (torch.empty_like(rm), torch.empty_like(rv), torch.empty_like(nb))
        if not (tr and tk and rm.numel()):
            dsts += list(o)
            srcs += [rm, rv, nb]
        outs.append(o)
    _copy_many(dsts, srcs)
    return outs


# ------------------------------------------------------------------- knn ----
@torch.library.custom_op("dgx::knn", mutates_args=(), device_types="cuda")
def knn(x: Tensor, k: int) -> Tensor:
    """int64 (B, N, k) local ids of the k nearest points (reference dgcnn.py:6-12)."""
    return ops.knn(x, k).clone() if getattr(ops._tls, "cache", None) is not None else ops.knn(x, k)


@knn.register_kernel("cpu")
def _(x, k):
    return cpu.knn(x, k)


@knn.register_fake
def _(x, k):
    B, _, N = x.shape
    return x.new_empty((B, N, k), dtype=torch.int64)


# distances are computed in fp32 whatever autocast says
torch.library.register_autocast("dgx::knn", "cuda", torch.float32)


# --------------------------------------------------------- graph feature ----
def _gf_shape(x, k, mode):
    B, C, N = x.shape
    if mode in (ops.nat.GF_CAT, ops.nat.GF_DIFFCAT):
        return (B, 2 * C, N, k)
    if mode == ops.nat.GF_DISP:
        return (B, C, N, k)
    return (B, N, k, C)


@torch.library.custom_op("dgx::graph_feature", mutates_args=(), device_types="cuda")
def graph_feature(x: Tensor, k: int, mode: int) -> tuple[Tensor, Tensor]:
    """(edge tensor, int32 kNN ids) of reference dgcnn.py:15-44; mode 0 =
    cat(x_j, x_i) (B,2C,N,k), 1 = x_j - x_i (B,C,N,k), 2 = x_j (B,N,k,C)."""
    xf = x.float()
    idx = ops.knn_raw(xf.detach(), k, out_dtype=_I32)
    shared = idx._base is not None or getattr(ops._tls, "cache", None) is not None   # a cache entry: never alias it
    return ops._GraphFeature.forward(_Rec(), xf, idx, mode), idx.clone() if shared else idx


@graph_feature.register_kernel("cpu")
def _(x, k, mode):
    xf = x.float().detach()
    idx = cpu.knn(xf, k)
    out = cpu.graph_feature(xf, k, knn_only=mode == ops.nat.GF_KNN_ONLY, disp_only=mode == ops.nat.GF_DISP, idx=idx,
                            mode="diff" if mode == ops.nat.GF_DIFFCAT else "cat")
    return out, idx.to(_I32)


@graph_feature.register_fake
def _(x, k, mode):
    B, _, N = x.shape
    return x.new_empty(_gf_shape(x, k, mode), dtype=_F32), x.new_empty((B, N, k), dtype=_I32)


@torch.library.custom_op("dgx::graph_feature_backward", mutates_args=(), device_types="cuda")
def graph_feature_backward(grad: Tensor, idx: Tensor, C: int, mode: int) -> Tensor:
    rec = _Rec()
    rec.saved_tensors = (idx,)
    rec.mode = mode
    B, N, _ = idx.shape
    rec.shape = (B, C, N)
    return ops._GraphFeature.backward(rec, grad)[0]


@graph_feature_backward.register_kernel("cpu")
def _(grad, idx, C, mode):
    """dx of the edge tensor (reference dgcnn.py:31-44 autograd): neighbour
    channels scatter-add to x_j, centre channels sum over k into x_i."""
    B, N, k = idx.shape
    flat = (idx.long() + torch.arange(B).view(-1, 1, 1) * N).view(-1)
    if mode == ops.nat.GF_KNN_ONLY:                       # (B, N, k, C) = x_j
        gn, gc = grad.reshape(B * N * k, C), None
    elif mode == ops.nat.GF_DISP:                         # (B, C, N, k) = x_j - x_i
        g = grad.permute(0, 2, 3, 1).reshape(B * N * k, C)
        gn, gc = g, -g
    elif mode == ops.nat.GF_DIFFCAT:                      # (B, 2C, N, k) = cat(x_j - x_i, x_i)
        g = grad.permute(0, 2, 3, 1).reshape(B * N * k, 2 * C)
        gn, gc = g[:, :C], g[:, C:] - g[:, :C]
    else:                                                 # (B, 2C, N, k) = cat(x_j, x_i)
        g = grad.permute(0, 2, 3, 1).reshape(B * N * k, 2 * C)
        gn, gc = g[:, :C], g[:, C:]
    rows = torch.zeros((B * N, C), dtype=torch.float32)
    rows.index_add_(0, flat, gn.float())
    if gc is not None:
        rows += gc.float().reshape(B * N, k, C).sum(dim=1)
    return rows.view(B, N, C).permute(0, 2, 1).contiguous()


@graph_feature_backward.register_fake
def _(grad, idx, C, mode):
    B, N, _ = idx.shape
    return grad.new_empty((B, C, N), dtype=_F32)


def _gf_setup(ctx, inputs, output):
    ctx.set_materialize_grads(False)   # no zero-filled gradients for the idx output
    ctx.save_for_backward(output[1])
    ctx.C, ctx.mode = inputs[0].shape[1], inputs[2]


def _gf_bwd(ctx, gout, _gidx):
    (idx,) = ctx.saved_tensors
    if gout is None:
        return None, None, None
    return torch.ops.dgx.graph_feature_backward(gout.contiguous(), idx, ctx.C, ctx.mode), None, None


torch.library.register_autograd("dgx::graph_feature", _gf_bwd, setup_context=_gf_setup)
torch.library.register_autocast("dgx::graph_feature", "cuda", torch.float32)


# ------------------------------------------------------------ weight prep ----
@torch.library.custom_op("dgx::weight_prep", mutates_args=(), device_types="cuda")
def weight_prep(weights: list[Tensor], rows: list[int], cols: list[int], stacked: list[bool],
                split: list[bool]) -> Tensor:
    """One bf16 buffer holding every weight's GEMM operand copies
    (gemm.prep_layout: [W | W_hi W_lo] and W^T per weight), one launch."""
    shapes = list(zip(rows, cols, stacked, split))
    total, _ = G.prep_layout(shapes)
    buf = torch.empty(total, dtype=_BF16, device=weights[0].device)
    G.prep_weights([(w.detach(), r, c, st, sp) for w, (r, c, st, sp) in zip(weights, shapes)], buf=buf)
    return buf


@weight_prep.register_fake
def _(weights, rows, cols, stacked, split):
    total, _ = G.prep_layout(list(zip(rows, cols, stacked, split)))
    return weights[0].new_empty((total,), dtype=_BF16)


def _dgcnn_prep_shapes(weights5):
    """(rows, cols, stacked, split) of DGCNN's bf16 copies: conv2-4 stacked and
    split (edgeconv), conv5 plain (models.dgcnn._bf16_weight_copies)."""
    shapes = [(w.shape[0], w.shape[1] // 2, True, True) for w in weights5[:3]]
    shapes.append((weights5[3].shape[0], weights5[3].shape[1], False, False))
    return shapes


# --------------------------------------------------------- edgeconv chain ----
_PER_LAYER = 9   # idx, PQ, ysel, arg, sumP, scale, shift, mean, invstd


def _chain_layers(weights, specs, slopes):
    return [E._Layer(w.shape[1] // 2, w.shape[0], s, sl) for w, s, sl in zip(weights, specs, slopes)]


@torch.library.custom_op("dgx::edgeconv_chain", mutates_args=(), device_types="cuda")
def edgeconv_chain(x: Tensor, k: int, weights: list[Tensor], gammas: list[Tensor], betas: list[Tensor],
                   running_means: list[Tensor], running_vars: list[Tensor], nbts: list[Tensor], training: list[bool],
                   track: list[bool], momentum: list[float], eps: list[float], slopes: list[float], bf16: bool,
                   need_grad: bool, prep: Optional[Tensor]) -> tuple[Tensor, Tensor, list[Tensor], list[Tensor],
                                                                     list[Tensor], list[Tensor]]:
    """DGCNN's EdgeConv blocks (dgcnn.py:84-100) on the C++ schedule
    (dgx_host::chain_forward): returns (concat buffer (B*N, sum Co), its bf16
    twin or empty, updated running means / vars / batch counters, the state the
    backward reads)."""
    from . import host
    host.load()
    outs = _stat_outputs(training, track, running_means, running_vars, nbts)
    rms, rvs, nbs = [o[0] for o in outs], [o[1] for o in outs], [o[2] for o in outs]
    specs = [_BNSpec(*a, out=o) for a, o in zip(zip(training, track, running_means, running_vars, nbts, momentum, eps),
                                                  outs)]
    bn_t, bn_f, bn_i, groups, sl = E._bn_lists(_chain_layers(weights, specs, slopes))
    idx0 = None
    if getattr(ops._tls, "cache", None) is not None:
        idx0 = ops.knn_raw(x.detach().float(), k, order=ops.reduction_order(x), out_dtype=_I32)
    xcat, xcat16, saved, _ = torch.ops.dgx_host.chain_forward(
        x.float(), k, weights, gammas, betas, bn_t, bn_f, bn_i, groups, sl, bf16, need_grad, prep, idx0, E.opts())
    saved = list(saved)
    x_pm = saved[0]
    if x_pm.untyped_storage().data_ptr() == x.untyped_storage().data_ptr():
        saved[0] = x_pm.clone()
    if idx0 is not None and saved[1].data_ptr() == idx0.data_ptr():
        saved[1] = idx0.clone()   # a cache entry: never alias it
    return xcat, xcat16, rms, rvs, nbs, saved


@edgeconv_chain.register_fake
def _(x, k, weights, gammas, betas, running_means, running_vars, nbts, training, track, momentum, eps, slopes,
      bf16, need_grad, prep):
    B, C0, N = x.shape
    M = B * N
    widths = [w.shape[0] for w in weights]
    total = sum(widths)
    selecting = [_use_batch(t, rm) or need_grad for t, rm in zip(training, running_means)]
    xcat = x.new_empty((M, total), dtype=_F32)
    xcat16 = x.new_empty((M, total), dtype=_BF16) if (bf16 and selecting[-1]) else x.new_empty((0,), dtype=_BF16)
    saved = [x.new_empty((M, C0), dtype=_F32)]
    for li, co in enumerate(widths):
        if not selecting[li]:
            saved += [x.new_empty((0,), dtype=_F32) for _ in range(_PER_LAYER)]
            continue
        saved += [x.new_empty((B, N, k), dtype=_I32), x.new_empty((M, 2 * co), dtype=_F32),
                  x.new_empty((M, co), dtype=_F32), x.new_empty((M, co), dtype=torch.uint8),
                  x.new_empty((M, co), dtype=_F32)] + [x.new_empty((co,), dtype=_F32) for _ in range(4)]
    return (xcat, xcat16, [torch.empty_like(t) for t in running_means], [torch.empty_like(t) for t in running_vars],
            [torch.empty_like(t) for t in nbts], saved)


@torch.library.custom_op("dgx::edgeconv_chain_backward", mutates_args=(), device_types="cuda")
def edgeconv_chain_backward(dxcat: Tensor, x: Tensor, xcat: Tensor, xcat16: Tensor, saved: list[Tensor],
                            weights: list[Tensor], gammas: list[Tensor], betas: list[Tensor], prep: Optional[Tensor],
                            k: int, use_batch: list[bool], slopes: list[float], bf16: bool,
                            x_needs_grad: bool) -> tuple[Tensor, list[Tensor], list[Tensor], list[Tensor]]:
    B, C0, N = x.shape
    dx, dws, dgs, dbs = torch.ops.dgx_host.chain_backward(
        dxcat, xcat, xcat16, saved, weights, prep, [B, C0, N], k, [int(not u) for u in use_batch],
        [""] * len(weights), slopes, bf16, x_needs_grad, E.opts())
    dx = dx.contiguous() if dx.numel() else _empty(x.device)
    return dx, [g.contiguous() for g in dws], list(dgs), list(dbs)


@edgeconv_chain_backward.register_fake
def _(dxcat, x, xcat, xcat16, saved, weights, gammas, betas, prep, k, use_batch, slopes, bf16, x_needs_grad):
    dx = x.new_empty(x.shape, dtype=_F32) if x_needs_grad else x.new_empty((0,), dtype=_F32)
    return (dx, [torch.empty_like(w, dtype=_F32) for w in weights], [torch.empty_like(g, dtype=_F32) for g in gammas],
            [torch.empty_like(b, dtype=_F32) for b in betas])


def _chain_setup(ctx, inputs, output):
    (x, k, weights, gammas, betas, rms, rvs, nbts, training, track, momentum, eps, slopes, bf16, need_grad,
     prep) = inputs
    xcat, xcat16, _, _, _, saved = output
    # the running statistics and saved-state outputs take no gradient: without
    # this autograd would zero-fill one gradient per saved tensor every step
    ctx.set_materialize_grads(False)
    ctx.n, ctx.nsaved, ctx.has_prep = len(weights), len(saved), prep is not None
    ctx.k, ctx.slopes, ctx.bf16 = k, list(slopes), bf16
    ctx.use_batch = [_use_batch(t, rm) for t, rm in zip(training, rms)]
    ctx.save_for_backward(x, xcat, xcat16, *saved, *weights, *gammas, *betas, *([prep] if prep is not None else []))


def _chain_bwd(ctx, g_xcat, _g16, _grm, _grv, _gnbt, _gsaved):
    t = ctx.saved_tensors
    n, ns = ctx.n, ctx.nsaved
    x, xcat, xcat16 = t[0], t[1], t[2]
    saved = list(t[3:3 + ns])
    ws, gs, bs = list(t[3 + ns:3 + ns + n]), list(t[3 + ns + n:3 + ns + 2 * n]), list(t[3 + ns + 2 * n:3 + ns + 3 * n])
    prep = t[3 + ns + 3 * n] if ctx.has_prep else None
    if g_xcat is None:
        g_xcat = torch.zeros_like(xcat)
    dx, dws, dgs, dbs = torch.ops.dgx.edgeconv_chain_backward(
        g_xcat.contiguous(), x, xcat, xcat16, saved, ws, gs, bs, prep, ctx.k, ctx.use_batch, ctx.slopes, ctx.bf16,
        ctx.needs_input_grad[0])
    nl = [None] * n   # list-of-tensor inputs take a list of gradients (none for the BN buffers)
    return ((dx if ctx.needs_input_grad[0] else None), None, dws, dgs, dbs, nl, list(nl), list(nl), None, None, None,
            None, None, None, None, None)


torch.library.register_autograd("dgx::edgeconv_chain", _chain_bwd, setup_context=_chain_setup)


# -------------------------------------------------------------- pointconv ----
def _pc_lds(bf16, X16, K):
    return bf16 and X16.numel() > 0 and K % 64 == 0


def _pc_prep(prep, Co, K):
    """conv5's (nt, tn) bf16 views of a weight-prep buffer, or (None, None)."""
    if prep is not None and prep.numel() == 2 * Co * K:
        return G.prep_views(prep, [(Co, K, False, False)])[0]
    return None, None


@torch.library.custom_op("dgx::pointconv", mutates_args=(), device_types="cuda")
def pointconv(X: Tensor, X16: Tensor, B: int, N: int, weight: Tensor, gamma: Tensor, beta: Tensor,
              running_mean: Tensor, running_var: Tensor, nbt: Tensor, training: bool, track: bool, momentum: float,
              eps: float, slope: float, bf16: bool, prep: Optional[Tensor]) -> tuple[Tensor, Tensor, Tensor, Tensor,
                                                                                    list[Tensor]]:
    """conv5 -> BN -> LeakyReLU on the concat buffer (dgcnn.py:100-102) on the
    C++ schedule (dgx_host::pointconv_forward): (out (B, Co, N), updated
    running mean / var / batch counter, saved state [Z, scale, shift, mean,
    invstd])."""
    from . import host
    host.load()
    (rm, rv, nb), = _stat_outputs([training], [track], [running_mean], [running_var], [nbt])
    spec = _BNSpec(training, track, running_mean, running_var, nbt, momentum, eps, out=(rm, rv, nb))
    t, f, i, g = bn_.op_args(spec)
    nt, tn = _pc_prep(prep, weight.shape[0], weight.shape[1])
    out, saved = torch.ops.dgx_host.pointconv_forward(X.float(), X16, B, N, weight, gamma, beta, t, f + [float(slope)],
                                                      i, g, bf16, nt, tn, E.opts())
    return out, rm, rv, nb, list(saved[1:6])


@pointconv.register_fake
def _(X, X16, B, N, weight, gamma, beta, running_mean, running_var, nbt, training, track, momentum, eps, slope,
      bf16, prep):
    M, K = X.shape
    Co = weight.shape[0]
    z16 = _pc_lds(bf16, X16, K) and _use_batch(training, running_mean)
    Z = X.new_empty((M, Co), dtype=_BF16 if z16 else _F32)
    return (X.new_empty((B, Co, N), dtype=_F32), torch.empty_like(running_mean), torch.empty_like(running_var),
            torch.empty_like(nbt), [Z] + [X.new_empty((Co,), dtype=_F32) for _ in range(4)])


@torch.library.custom_op("dgx::pointconv_backward", mutates_args=(), device_types="cuda")
def pointconv_backward(dout: Tensor, X: Tensor, X16: Tensor, weight: Tensor, saved: list[Tensor],
                       prep: Optional[Tensor], B: int, N: int, slope: float, bf16: bool,
                       use_batch: bool) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    M, K = X.shape
    Co = weight.shape[0]
    lds = _pc_lds(bf16, X16, K)
    e16 = torch.empty(0, dtype=_BF16, device=X.device)
    nt, tn = (_pc_prep(prep, Co, K) if lds else (None, None))
    if lds and nt is None:
        nt, tn = G.prep_weight(weight, Co, K, False)
    # fp32 mode: the backward op rebuilds the split-bf16 planes and weights from X
    full = [X16 if lds else X.float(), *saved, nt if lds else e16, tn if lds else e16, e16, e16]
    dX, dW, dg, db = torch.ops.dgx_host.pointconv_backward(dout, full, weight, B, N, slope, not use_batch, "", bf16,
                                                           E.opts())
    return dX.contiguous(), dW.contiguous(), dg, db


@pointconv_backward.register_fake
def _(dout, X, X16, weight, saved, prep, B, N, slope, bf16, use_batch):
    Co = weight.shape[0]
    return (X.new_empty(X.shape, dtype=_F32), torch.empty_like(weight, dtype=_F32), X.new_empty((Co,), dtype=_F32),
            X.new_empty((Co,), dtype=_F32))


def _pc_setup(ctx, inputs, output):
    (X, X16, B, N, weight, gamma, beta, rm, rv, nbt, training, track, momentum, eps, slope, bf16, prep) = inputs
    ctx.set_materialize_grads(False)
    ctx.meta = (B, N, slope, bf16, _use_batch(training, rm), prep is not None)
    ctx.save_for_backward(X, X16, weight, *output[4], *([prep] if prep is not None else []))


def _pc_bwd(ctx, g_out, _grm, _grv, _gnb, _gsaved):
    B, N, slope, bf16, use_batch, has_prep = ctx.meta
    t = ctx.saved_tensors
    X, X16, weight = t[0], t[1], t[2]
    saved = list(t[3:8])
    prep = t[8] if has_prep else None
    if g_out is None:
        g_out = torch.zeros((B, weight.shape[0], N), dtype=torch.float32, device=X.device)
    dX, dW, dg, db = torch.ops.dgx.pointconv_backward(g_out.contiguous(), X, X16, weight, saved, prep, B, N, slope,
                                                      bf16, use_batch)
    return dX, None, None, None, dW, dg, db, None, None, None, None, None, None, None, None, None, None


torch.library.register_autograd("dgx::pointconv", _pc_bwd, setup_context=_pc_setup)


# ------------------------------------------------------------------ DGCNN ----
def _bn_args(bn, dev):
    e = _empty(dev)
    return (bn.running_mean if bn.running_mean is not None else e,
            bn.running_var if bn.running_var is not None else e,
            bn.num_batches_tracked if bn.num_batches_tracked is not None else _empty(dev, torch.int64),
            bn.training, bn.track_running_stats, -1.0 if bn.momentum is None else float(bn.momentum), float(bn.eps))


def _store_bn(pairs):
    """Copy the ops' updated running statistics into the modules (only where
    nn.BatchNorm would have updated them: training and tracking), all layers in
    one multi-tensor copy per dtype. ``pairs``: (bn, rm, rv, nbt) per layer."""
    dsts, srcs = [], []
    for bn, rm, rv, nb in pairs:
        if not bn_.mode(bn)[1]:
            continue
        for d, s in ((bn.running_mean, rm), (bn.running_var, rv), (bn.num_batches_tracked, nb)):
            if d is not None:
                dsts.append(d)
                srcs.append(s)
    with torch.no_grad():
        _copy_many(dsts, srcs)


def enabled_for(model):
    """The op path (torch.compile / export) serves a model whose BatchNorms are
    plain nn.BatchNorm (a process group cannot cross a traced op's boundary)."""
    return ENABLED and not any(isinstance(m, torch.nn.SyncBatchNorm) for m in model.modules())


def dgcnn_forward(model, x):
    """models.dgcnn.DGCNN.forward through torch.ops.dgx (dgcnn.py:80-103)."""
    ops.nat.require_device(x)   # no CPU fallback: a CPU cloud fails loudly here
    B, _, N = x.shape
    x = x.float()
    dev = x.device
    bf16 = prec.effective() == "bf16"
    blocks = model.edge_blocks()
    convs = [b[0] for b in blocks]
    bns = [b[1] for b in blocks]
    c5, bn5, act5 = model.conv5[0], model.conv5[1], model.conv5[2]
    for conv, bn in zip(convs + [c5], bns + [bn5]):
        if conv.bias is not None or bn.weight is None:
            raise NotImplementedError("dgx DGCNN expects Conv(bias=False) + affine BatchNorm (dgcnn.py:54-78)")
    eff = model.edge_weights()   # per-block conv weights (re-parameterised in edge_mode "diff")
    params = [p for w, bn in zip(eff + [c5.weight], bns + [bn5]) for p in (w, bn.weight, bn.bias)]
    need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
    prep = None
    if bf16:   # one launch for every bf16 operand copy of the step (blocks 2-4, conv5)
        ws = [w.detach() for w in eff[1:]] + [c5.weight.detach()]
        shapes = _dgcnn_prep_shapes(ws)
        prep = torch.ops.dgx.weight_prep(ws, [s[0] for s in shapes], [s[1] for s in shapes],
                                         [s[2] for s in shapes], [s[3] for s in shapes])
    bn_in = [_bn_args(bn, dev) for bn in bns]
    xcat, xcat16, rms, rvs, nbs, _ = torch.ops.dgx.edgeconv_chain(
        x, model.k, eff, [bn.weight for bn in bns], [bn.bias for bn in bns],
        [a[0] for a in bn_in], [a[1] for a in bn_in], [a[2] for a in bn_in], [a[3] for a in bn_in],
        [a[4] for a in bn_in], [a[5] for a in bn_in], [a[6] for a in bn_in],
        [float(b[2].negative_slope) for b in blocks], bf16, need_grad, prep)
    a5 = _bn_args(bn5, dev)
    prep5 = None
    if prep is not None:
        # conv5's copies are the last entry of the shared buffer: pass them as their own view
        _, lay = G.prep_layout(_dgcnn_prep_shapes(eff[1:] + [c5.weight]))
        off = lay[3][0]
        prep5 = prep[off:]
    out, rm5, rv5, nb5, _ = torch.ops.dgx.pointconv(xcat, xcat16, B, N, c5.weight, bn5.weight, bn5.bias, a5[0], a5[1],
                                                     a5[2], a5[3], a5[4], a5[5], a5[6], float(act5.negative_slope),
                                                     bf16, prep5)
    _store_bn(list(zip(bns, rms, rvs, nbs)) + [(bn5, rm5, rv5, nb5)])
    return out


# ------------------------------------------------- PositionEmbedding edge MLP ----
# dgx::edge_mlp2: PositionEmbedding's edge stage (reference models/layers.py:
# 45-52: get_graph_feature -> conv1 -> conv2 -> max over k) as dgx.edgemlp runs
# it. The forward returns the output and the updated BatchNorm statistics only;
# the backward op re-runs the forward kernels (no statistics update: the BNs
# are replayed with their batch / running choice and tracking off) to rebuild
# the saved state, then runs the engine's backward — the same kernels on the
# same inputs, so the gradients equal the eager Function path's bit for bit.
# Eager callers keep the Function path (no recompute); torch.compile / export
# trace this op (dgx.edgemlp.edge_mlp2 routes here while compiling).
def _emlp_specs(training, track, rms, rvs, nbts, momentum, eps, outs):
    return [_BNSpec(t, tr, rm, rv, nb, mo, e, out=o)
            for t, tr, rm, rv, nb, mo, e, o in zip(training, track, rms, rvs, nbts, momentum, eps, outs)]


@torch.library.custom_op("dgx::edge_mlp2", mutates_args=(), device_types="cuda")
def edge_mlp2(x: Tensor, k: int, w1: Tensor, g1: Tensor, b1: Tensor, rm1: Tensor, rv1: Tensor, nbt1: Tensor,
              w2: Tensor, g2: Tensor, b2: Tensor, rm2: Tensor, rv2: Tensor, nbt2: Tensor, training: list[bool],
              track: list[bool], momentum: list[float], eps: list[float], slopes: list[float], bf16: bool,
              knn_src: Optional[Tensor]) -> tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    from . import edgemlp as EM
    outs = _stat_outputs(training, track, [rm1, rm2], [rv1, rv2], [nbt1, nbt2])
    s1, s2 = _emlp_specs(training, track, [rm1, rm2], [rv1, rv2], [nbt1, nbt2], momentum, eps, outs)
    with prec.mode("bf16" if bf16 else "fp32"):
        out = EM._EdgeMLP2.forward(_Rec(), x, k, s1, s2, slopes[0], slopes[1], False, knn_src, bf16, w1, g1, b1, w2,
                                   g2, b2)
    (a1, a2, a3), (c1, c2, c3) = outs
    return out, a1, a2, a3, c1, c2, c3


@edge_mlp2.register_fake
def _(x, k, w1, g1, b1, rm1, rv1, nbt1, w2, g2, b2, rm2, rv2, nbt2, training, track, momentum, eps, slopes, bf16,
      knn_src):
    B, _, N = x.shape
    return (x.new_empty((B, w2.shape[0], N), dtype=_F32), torch.empty_like(rm1), torch.empty_like(rv1),
            torch.empty_like(nbt1), torch.empty_like(rm2), torch.empty_like(rv2), torch.empty_like(nbt2))


@torch.library.custom_op("dgx::edge_mlp2_backward", mutates_args=(), device_types="cuda")
def edge_mlp2_backward(dout: Tensor, x: Tensor, k: int, w1: Tensor, g1: Tensor, b1: Tensor, rm1: Tensor, rv1: Tensor,
                       w2: Tensor, g2: Tensor, b2: Tensor, rm2: Tensor, rv2: Tensor, use_batch: list[bool],
                       eps: list[float], slopes: list[float], bf16: bool, knn_src: Optional[Tensor],
                       x_needs_grad: bool) -> tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    from . import edgemlp as EM
    e = _empty(x.device)
    en = _empty(x.device, torch.int64)
    specs = [_BNSpec(u, False, rm if not u else e, rv if not u else e, en, 0.1, ep)
             for u, rm, rv, ep in zip(use_batch, (rm1, rm2), (rv1, rv2), eps)]
    rec = _Rec()
    rec.needs_input_grad = (x_needs_grad,) + (True,) * 63
    with prec.mode("bf16" if bf16 else "fp32"):
        EM._EdgeMLP2.forward(rec, x, k, specs[0], specs[1], slopes[0], slopes[1], True, knn_src, bf16, w1, g1, b1,
                             w2, g2, b2)
        res = EM._EdgeMLP2.backward(rec, dout)
    dx = res[0].contiguous() if res[0] is not None else _empty(x.device)
    gw1, dg1, db1, gw2, dg2, db2 = res[9:15]
    return dx, gw1.contiguous(), dg1, db1, gw2.contiguous(), dg2, db2


@edge_mlp2_backward.register_fake
def _(dout, x, k, w1, g1, b1, rm1, rv1, w2, g2, b2, rm2, rv2, use_batch, eps, slopes, bf16, knn_src, x_needs_grad):
    dx = x.new_empty(x.shape, dtype=_F32) if x_needs_grad else x.new_empty((0,), dtype=_F32)
    return (dx, torch.empty_like(w1, dtype=_F32), torch.empty_like(g1, dtype=_F32), torch.empty_like(b1, dtype=_F32),
            torch.empty_like(w2, dtype=_F32), torch.empty_like(g2, dtype=_F32), torch.empty_like(b2, dtype=_F32))


def _emlp_setup(ctx, inputs, output):
    (x, k, w1, g1, b1, rm1, rv1, nbt1, w2, g2, b2, rm2, rv2, nbt2, training, track, momentum, eps, slopes, bf16,
     knn_src) = inputs
    ctx.set_materialize_grads(False)
    ctx.k, ctx.eps, ctx.slopes, ctx.bf16 = k, list(eps), list(slopes), bf16
    ctx.use_batch = [_use_batch(training[0], rm1), _use_batch(training[1], rm2)]
    ctx.has_src = knn_src is not None
    # the recompute reads the running statistics only where they normalised the
    # forward (no batch statistics: then they are not updated either); a layer
    # on batch statistics saves nothing of them — its buffers get the op's
    # updated values copied in after the call (edge_mlp2_call), which would
    # invalidate a saved reference
    e = x.new_empty((0,), dtype=_F32)
    rms = [rm if not ub else e for rm, ub in zip((rm1, rm2), ctx.use_batch)]
    rvs = [rv if not ub else e for rv, ub in zip((rv1, rv2), ctx.use_batch)]
    ctx.save_for_backward(x, w1, g1, b1, rms[0], rvs[0], w2, g2, b2, rms[1], rvs[1],
                          *([knn_src] if ctx.has_src else []))


def _emlp_bwd(ctx, gout, *_stats):
    t = ctx.saved_tensors
    x, w1, g1, b1, rm1, rv1, w2, g2, b2, rm2, rv2 = t[:11]
    knn_src = t[11] if ctx.has_src else None
    if gout is None:
        gout = torch.zeros((x.shape[0], w2.shape[0], x.shape[2]), dtype=_F32, device=x.device)
    dx, gw1, dg1, db1, gw2, dg2, db2 = torch.ops.dgx.edge_mlp2_backward(
        gout, x, ctx.k, w1, g1, b1, rm1, rv1, w2, g2, b2, rm2, rv2, ctx.use_batch, ctx.eps, ctx.slopes, ctx.bf16,
        knn_src, ctx.needs_input_grad[0])
    return ((dx if ctx.needs_input_grad[0] else None), None, gw1, dg1, db1, None, None, None, gw2, dg2, db2, None,
            None, None, None, None, None, None, None, None, None)


torch.library.register_autograd("dgx::edge_mlp2", _emlp_bwd, setup_context=_emlp_setup)


def edge_mlp2_call(x, k, conv1, conv2, knn_src=None):
    """models.layers.PositionEmbedding's edge stage through dgx::edge_mlp2 (the
    module BatchNorms' buffers updated from the op's outputs)."""
    (cv1, bn1, act1), (cv2, bn2, act2) = (conv1[0], conv1[1], conv1[2]), (conv2[0], conv2[1], conv2[2])
    dev = x.device
    a1, a2 = _bn_args(bn1, dev), _bn_args(bn2, dev)
    out, rm1, rv1, nb1, rm2, rv2, nb2 = torch.ops.dgx.edge_mlp2(
        x.float(), k, cv1.weight, bn1.weight, bn1.bias, a1[0], a1[1], a1[2], cv2.weight, bn2.weight, bn2.bias, a2[0],
        a2[1], a2[2], [a1[3], a2[3]], [a1[4], a2[4]], [a1[5], a2[5]], [a1[6], a2[6]],
        [float(act1.negative_slope), float(act2.negative_slope)], prec.effective() == "bf16",
        None if knn_src is None else knn_src.detach().float())
    _store_bn([(bn1, rm1, rv1, nb1), (bn2, rm2, rv2, nb2)])
    return out


# -------------------------------------------------------------- attention ----
# dgx::attention: Net's attention core (reference models/model_partseg.py:
# 167-171, 187-191 via nn.MultiheadAttention): dropout(softmax(scale q k^T)) v
# per head on the engine kernels. The dropout seed is an input drawn by the
# caller on the device (dgx.attention.new_seed), so the op is a pure function
# of its inputs; the log-sum-exp comes back for the backward op.
@torch.library.custom_op("dgx::attention", mutates_args=(), device_types="cuda")
def attention_op(q: Tensor, k: Tensor, v: Tensor, heads: int, p: float, scale: float, dtype_code: int,
                 seed: Optional[Tensor]) -> tuple[Tensor, Tensor]:
    from . import attention as A
    return A.attn_forward(q, k, v, heads, p, scale, A.CODE_DTYPES[dtype_code], seed)


@attention_op.register_fake
def _(q, k, v, heads, p, scale, dtype_code, seed):
    from . import attention as A
    B, Nq, E = q.shape
    return q.new_empty((B, Nq, E), dtype=A.CODE_DTYPES[dtype_code]), q.new_empty((B * heads * Nq,), dtype=_F32)


@torch.library.custom_op("dgx::attention_backward", mutates_args=(), device_types="cuda")
def attention_backward(do: Tensor, q: Tensor, k: Tensor, v: Tensor, o: Tensor, lse: Tensor, heads: int, p: float,
                       scale: float, seed: Optional[Tensor]) -> tuple[Tensor, Tensor, Tensor]:
    from . import attention as A
    return A.attn_backward(do, q, k, v, o, lse, heads, p, scale, seed)


@attention_backward.register_fake
def _(do, q, k, v, o, lse, heads, p, scale, seed):
    return torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)


def _attn_setup(ctx, inputs, output):
    q, k, v, heads, p, scale, dtype_code, seed = inputs
    ctx.set_materialize_grads(False)
    ctx.meta = (heads, p, scale)
    ctx.save_for_backward(q, k, v, output[0], output[1], *([seed] if seed is not None else []))


def _attn_bwd(ctx, do, _glse):
    heads, p, scale = ctx.meta
    t = ctx.saved_tensors
    q, k, v, o, lse = t[:5]
    seed = t[5] if len(t) > 5 else None
    if do is None:
        return None, None, None, None, None, None, None, None
    dq, dk, dv = torch.ops.dgx.attention_backward(do, q, k, v, o, lse, heads, p, scale, seed)
    return dq, dk, dv, None, None, None, None, None


torch.library.register_autograd("dgx::attention", _attn_bwd, setup_context=_attn_setup)


# ---------------------------------------------------------------------- HOG ----
# dgx::hog_1x1: compute_hog_1x1 after its kNN call (reference
# models/model_partseg.py:28-92). No gradient (the reference detaches into numpy).
@torch.library.custom_op("dgx::hog_1x1", mutates_args=(), device_types="cuda")
def hog_1x1_op(x: Tensor, idx: Tensor) -> Tensor:
    from . import hog as H
    return H.hog_1x1(x, idx)


@hog_1x1_op.register_kernel("cpu")
def _(x, idx):
    return cpu.hog_1x1(x, idx)


@hog_1x1_op.register_fake
def _(x, idx):
    B, _, N = x.shape
    return x.new_empty((B, N, 18), dtype=_F32)
