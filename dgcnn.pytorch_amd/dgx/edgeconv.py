"""Fused EdgeConv stack: the DGCNN block chain of reference models/dgcnn.py:84-100.

Reference, per block l (dgcnn.py:84-98):
    e = get_graph_feature(x_{l-1}, k)                     (B, 2C, N, k)
    x_l = max_k LeakyReLU(BN(Conv2d_1x1(e)))               (B, Co, N)
and then cat(x1..x4) (dgcnn.py:100).

Engine: one autograd node for the whole chain. Activations live point-major in
ONE concat buffer xcat (B*N, sum Co) in HBM; block l reads its input as a
column slice of xcat and writes its output straight into its own slice, so the
torch.cat of dgcnn.py:100 is free. Per block:
    idx   = knn(x_{l-1})                      HIP (bit-exact with the reference)
    PQ    = X [W1; W2]^T                      (B*N, 2Co) per-point GEMM
    gather/finalize/apply                     HIP (edge max/min + BN stats + LReLU)
Backward per block (reverse order):
    dz, BN-bwd affine                         HIP
    reverse kNN graph + dPQ                   HIP
    dX += dPQ [W1; W2], dW = dPQ^T X          GEMM (accumulated into xcat's grad)
"""
import torch

from . import _native as nat
from . import dist as dist_
from . import gemm as G
from . import precision as prec
from .ops import knn_raw, reduction_order


# Optional capture for tests/tools: when a dict, forward stores each block's
# routing decisions (idx, arg, zpos) under ("fwd", l) and backward stores
# intermediates under l. Off (None) in normal use.
_debug = None


def _bn_factor(bn):
    """(exponential-average factor nn.BatchNorm uses this step, num_batches_tracked
    tensor for the finalize kernel to increment or None). With a momentum the
    counter is bumped on device by dgx_bn_finalize_f32 (no extra launch); the
    cumulative-average form (momentum None) needs the count on the host."""
    if bn.momentum is None:
        if bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
            return 1.0 / float(bn.num_batches_tracked.item()), None
        return 0.0, None
    return float(bn.momentum), bn.num_batches_tracked


def _reverse_graph(idx, B, N, k, dev):
    """Reverse kNN graph (CSR of in-edges, dgx_graph_reverse) of one block, on
    the current stream. Built in the backward, right before its consumer: a
    build on a side stream overlapping the forward measured slower (1.63 vs
    1.56 ms/step at cfg2; the concurrent kernels contend for the L2 the kNN
    operand images live in)."""
    M = B * N
    rowptr = torch.empty(M + 1, dtype=torch.int32, device=dev)
    edges = torch.empty(M * k, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        nat.check(nat.lib().dgx_graph_reverse(nat.ptr(idx), B, N, k, nat.ptr(rowptr), nat.ptr(edges),
                                              nat.stream_of(idx)), "reverse graph")
    return rowptr, edges


class _Layer:
    """Non-tensor description of one block (weights are passed as tensors)."""

    def __init__(self, cin, cout, bn, slope):
        self.cin, self.cout, self.bn, self.slope = cin, cout, bn, slope


def _split_weight(w, cin, cout):
    w = w.reshape(cout, 2 * cin)
    # rows [0,Co) produce P (neighbour half, channels [0,C)), rows [Co,2Co) Q (centre half)
    return torch.cat([w[:, :cin], w[:, cin:]], dim=0)


class _EdgeConvStack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, layers, training, ctx_preps, *params):
        dev = x.device
        B, C0, N = x.shape
        M = B * N
        widths = [ly.cout for ly in layers]
        total = sum(widths)
        L = nat.lib()
        stream = nat.stream_of(x)
        bf16 = prec.get() == "bf16"
        xcat = torch.empty((M, total), dtype=torch.float32, device=dev)
        # bf16 twin of the concat buffer: the GEMM operand copy, written by the
        # same kernel that writes xcat (precision "bf16" only)
        xcat16 = torch.empty((M, total), dtype=torch.bfloat16, device=dev) if bf16 else None
        x_pm = x.permute(0, 2, 1).reshape(M, C0)  # point-major input rows (copy only if needed)
        saved = []
        off_in = None
        count = float(M * k)
        have16 = False  # xcat16 holds the previous block's output
        # bf16 [W1;W2] and transposed copies of blocks 2.. in one launch (used when
        # the block's input is the bf16 twin, i.e. after a batch-statistics block)
        preps = list(ctx_preps) if ctx_preps is not None else [None] * len(layers)
        if bf16 and len(layers) > 1 and ctx_preps is None:
            jobs = [(params[3 * li], ly.cout, ly.cin, True) for li, ly in enumerate(layers) if li > 0]
            preps[1:] = G.prep_weights(jobs)
        for li, ly in enumerate(layers):
            w, gamma, beta = params[3 * li: 3 * li + 3]
            cin, co = ly.cin, ly.cout
            if li == 0:
                X = x_pm
                idx = knn_raw(x, k, order=reduction_order(x), out_dtype=torch.int32)
            else:
                X = xcat[:, off_in:off_in + cin]
                # the reference's blocks 2-4 see contiguous (B,C,N) features (max over
                # dim -1 of a contiguous tensor), hence the strided rounding order
                idx = knn_raw(xcat[:, off_in:], k, order=nat.ORDER_STRIDED, out_dtype=torch.int32,
                              strides=(N * total, 1, total), shape=(B, cin, N))
            wprep = None
            if bf16:
                X16 = xcat16[:, off_in:off_in + cin] if li > 0 else None
                if have16 and G.lds_ok_nt(X16, cin):
                    # bf16 operands by LDS-DMA; the weight's bf16 [W1;W2] and transpose serve fwd and bwd
                    wprep = preps[li]
                    PQ = G.lds_xwt(X16, wprep[0])
                else:
                    PQ = G.mm_xwt(X, _split_weight(w, cin, co))  # fp32 operands rounded while staged
            else:
                PQ = prec.mm(X, _split_weight(w, cin, co).t())
            off = sum(widths[:li])
            out = xcat[:, off:off + co]
            bn = ly.bn
            use_batch = training or bn.running_mean is None
            scale = torch.empty(co, dtype=torch.float32, device=dev)
            shift = torch.empty_like(scale)
            with torch.cuda.device(dev):
                if use_batch:
                    ysel = torch.empty((M, co), dtype=torch.float32, device=dev)
                    arg = torch.empty((M, co), dtype=torch.uint8, device=dev)
                    sumP = torch.empty((M, co), dtype=torch.float32, device=dev)
                    prow = L.dgx_edge_partials_rows(B, N, co)
                    partials = torch.empty((prow, 2, co), dtype=torch.float32, device=dev)
                    mean = torch.empty_like(scale)
                    invstd = torch.empty_like(scale)
                    nat.check(L.dgx_edge_fwd_gather_f32(
                        nat.ptr(PQ), 2 * co, nat.ptr(idx), B, N, k, co, nat.ptr(gamma), nat.ptr(ysel),
                        nat.ptr(arg), nat.ptr(sumP), nat.ptr(partials), prow, stream), "edge gather")
                    update = training and bn.running_mean is not None
                    factor, nbt = _bn_factor(bn) if update else (0.0, None)
                    fin, frows, fcount = partials, prow, count
                    sync, group = dist_.sync_group(bn, training)
                    if sync:  # SyncBatchNorm: statistics of the global batch, one all-reduce
                        tot, fcount = dist_.allreduce_sums(partials.sum(0), count, group)
                        fin, frows = tot.unsqueeze(0).contiguous(), 1
                    nat.check(L.dgx_bn_finalize_f32(
                        nat.ptr(fin), frows, co, fcount, nat.ptr(gamma), nat.ptr(beta),
                        nat.ptr(bn.running_mean) if update else None,
                        nat.ptr(bn.running_var) if update else None, factor, float(bn.eps),
                        nat.ptr(scale), nat.ptr(shift), nat.ptr(mean), nat.ptr(invstd), nat.ptr(nbt), stream),
                        "bn finalize")
                    out16 = xcat16[:, off:off + co] if bf16 else None
                    nat.check(L.dgx_bn_lrelu_apply_f32(nat.ptr(ysel), M, co, nat.ptr(scale), nat.ptr(shift),
                                                       float(ly.slope), nat.ptr(out), total, nat.ptr(out16), stream),
                              "bn apply")
                    have16 = bf16
                    saved.append((idx, PQ, ysel, arg, sumP, scale, shift, mean, invstd, wprep,
                                  group if sync else None))
                    if _debug is not None:
                        # sign of fmaf(scale, ysel, shift) as the kernels evaluate it: the fp64
                        # product of two fp32 values is exact, so this sign is fma's sign
                        zpos = (scale.double() * ysel.double() + shift.double()) > 0
                        _debug[("fwd", li)] = (idx.clone(), arg.clone(), zpos)
                else:
                    nat.check(L.dgx_bn_eval_affine_f32(
                        co, nat.ptr(gamma), nat.ptr(beta), nat.ptr(bn.running_mean), nat.ptr(bn.running_var),
                        float(bn.eps), nat.ptr(scale), nat.ptr(shift), stream), "bn eval affine")
                    nat.check(L.dgx_edge_fwd_eval_f32(
                        nat.ptr(PQ), 2 * co, nat.ptr(idx), B, N, k, co, nat.ptr(scale), nat.ptr(shift),
                        float(ly.slope), nat.ptr(out), total, stream), "edge eval")
                    have16 = False
                    saved.append(None)
            off_in = off
        ctx.k = k
        ctx.layers = layers
        ctx.shape = (B, C0, N)
        ctx.layer_state = saved
        ctx.x_needs_grad = x.requires_grad
        ctx.bf16 = bf16
        ctx.save_for_backward(x_pm, xcat, xcat16, *params)
        if xcat16 is None or not have16:
            xcat16 = torch.empty(0, dtype=torch.bfloat16, device=dev)
        ctx.mark_non_differentiable(xcat16)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the bf16 twin
        return xcat, xcat16

    @staticmethod
    def backward(ctx, dxcat, _unused):
        if dxcat is None:
            return (None,) * (5 + len(ctx.saved_tensors) - 3)
        if any(s is None for s in ctx.layer_state):
            raise RuntimeError("dgx EdgeConv: backward through an eval-mode (running-stats) forward is not supported")
        x_pm, xcat, xcat16, *params = ctx.saved_tensors
        layers, k = ctx.layers, ctx.k
        B, C0, N = ctx.shape
        M = B * N
        dev = xcat.device
        L = nat.lib()
        stream = nat.stream_of(xcat)
        widths = [ly.cout for ly in layers]
        total = sum(widths)
        bf16 = ctx.bf16
        grads = [None] * len(params)
        dx_in = None
        count = float(M * k)
        nl = len(layers)
        if bf16:
            # The incoming gradient stays read-only: block l's input gradient is written
            # as addend (incoming slice) + dPQ Wcat into a fresh buffer, no clone pass.
            dxcat = dxcat.contiguous()
            lead = total - widths[-1]
            dnew = torch.empty((M, max(lead, 1)), dtype=torch.float32, device=dev)
        else:
            dxcat = dxcat.contiguous().clone()
        for li in reversed(range(nl)):
            ly = layers[li]
            cin, co = ly.cin, ly.cout
            w = params[3 * li]
            idx, PQ, ysel, arg, sumP, scale, shift, mean, invstd, wprep, group = ctx.layer_state[li]
            rowptr, edges = _reverse_graph(idx, B, N, k, dev)
            off = sum(widths[:li])
            prev = off - widths[li - 1] if li > 0 else None
            X = x_pm if li == 0 else xcat[:, prev: prev + cin]
            if bf16 and li < nl - 1:
                dY, ldy = dnew[:, off:off + co], dnew.stride(0)
            else:
                dY, ldy = dxcat[:, off:off + co], dxcat.stride(0)
            nblk = max(1, min(1024, (M + 63) // 64))
            dz = torch.empty((M, co), dtype=torch.float32, device=dev)  # dz with packed slot
            partials = torch.empty((nblk, 2, co), dtype=torch.float32, device=dev)
            dgamma = torch.empty(co, dtype=torch.float32, device=dev)
            dbeta = torch.empty(co, dtype=torch.float32, device=dev)
            c0 = torch.empty(co, dtype=torch.float32, device=dev)
            c1 = torch.empty(co, dtype=torch.float32, device=dev)
            # dPQ only feeds the GEMMs: bf16 (what the GEMM would round it to) in bf16 mode
            dPQ = torch.empty((M, 2 * co), dtype=torch.bfloat16 if bf16 else torch.float32, device=dev)
            with torch.cuda.device(dev):
                nat.check(L.dgx_edge_bwd_dz_f32(
                    nat.ptr(dY), ldy, nat.ptr(ysel), nat.ptr(arg), M, co, nat.ptr(scale), nat.ptr(shift),
                    nat.ptr(mean), nat.ptr(invstd), float(ly.slope), nat.ptr(dz), nat.ptr(partials), nblk, stream),
                    "edge bwd dz")
                if group is None:
                    nat.check(L.dgx_bn_bwd_finalize_f32(
                        nat.ptr(partials), nblk, co, count, nat.ptr(scale), nat.ptr(mean), nat.ptr(invstd),
                        nat.ptr(dgamma), nat.ptr(dbeta), nat.ptr(c0), nat.ptr(c1), 0, stream), "bn bwd finalize")
                else:  # SyncBatchNorm: input gradient from global sums, gamma/beta grads rank-local
                    loc = partials.sum(0)
                    tot, gcount = dist_.allreduce_sums(loc, count, group)
                    tot = tot.unsqueeze(0).contiguous()
                    nat.check(L.dgx_bn_bwd_finalize_f32(
                        nat.ptr(tot), 1, co, gcount, nat.ptr(scale), nat.ptr(mean), nat.ptr(invstd),
                        None, None, nat.ptr(c0), nat.ptr(c1), 0, stream), "bn bwd finalize")
                    dbeta.copy_(loc[0])
                    dgamma.copy_(loc[1])
                nat.check(L.dgx_edge_bwd_scatter_f32(
                    nat.ptr(PQ), 2 * co, nat.ptr(rowptr), nat.ptr(edges), nat.ptr(dz), nat.ptr(sumP), B, N, k, co,
                    nat.ptr(scale), nat.ptr(c0), nat.ptr(c1), nat.ptr(dPQ), int(bf16), stream), "edge bwd scatter")
            if _debug is not None:
                _debug[li] = {"dY": dY.clone(), "dz": dz.clone(), "dgamma": dgamma.clone(), "dbeta": dbeta.clone(),
                              "c0": c0.clone(), "c1": c1.clone(), "dPQ": dPQ.float(), "partials": partials.clone(),
                              "ysel": ysel.clone(), "scale": scale.clone(), "shift": shift.clone(),
                              "arg": arg.clone(), "idx": idx.clone(), "PQ": PQ.clone(), "sumP": sumP.clone(),
                              "mean": mean.clone(), "invstd": invstd.clone(), "X": X.clone(),
                              "rowptr": rowptr.clone(), "edges": edges.clone()}
            grads[3 * li + 1] = dgamma
            grads[3 * li + 2] = dbeta
            if bf16:
                # dW = dPQ^T X, un-stacked to the reference layout [W1 | W2]
                gw = torch.empty((co, 2 * cin), dtype=torch.float32, device=dev)
                if wprep is not None:
                    G.lds_atb(dPQ, xcat16[:, prev:prev + cin], gw, split_rows=co)
                else:
                    G.mm_atb(dPQ, X, gw, split_rows=co)
                grads[3 * li] = gw.view(w.shape)
                if li > 0:
                    dst = dnew[:, prev:prev + cin]
                    add = dxcat[:, prev:prev + cin]
                    if wprep is not None:
                        G.lds_xwt(dPQ, wprep[1], out=dst, addend=add)
                    else:
                        dst.copy_(add)
                        G.mm_xw(dPQ, _split_weight(w, cin, co), out=dst, accumulate=True)
                elif ctx.x_needs_grad:
                    dx_in = G.mm_xw(dPQ, _split_weight(w, cin, co)).view(B, N, C0).permute(0, 2, 1)
            else:
                wcat = _split_weight(w, cin, co)
                dwcat = prec.mm(dPQ.t(), X)  # (2Co, C)
                grads[3 * li] = torch.cat([dwcat[:co], dwcat[co:]], dim=1).reshape(w.shape)
                if li > 0:
                    dxcat[:, prev:prev + cin] += prec.mm(dPQ, wcat)
                elif ctx.x_needs_grad:
                    dx_in = prec.mm(dPQ, wcat).view(B, N, C0).permute(0, 2, 1)
        return (dx_in, None, None, None, None, *grads)


def edgeconv_stack_pair(x, k, convs, training, preps=None):
    """As edgeconv_stack, also returning the bf16 twin of the concat buffer
    (empty unless precision "bf16" produced it): conv5's GEMM operand.
    ``preps``: optional per-block bf16 weight copies (gemm.prep_weights) made
    by the caller in one launch with other layers' (None for block 1)."""
    nat.require_device(x)
    if x.dtype != torch.float32:
        x = x.float()
    layers, params = [], []
    for seq in convs:
        conv, bn, act = seq[0], seq[1], seq[2]
        co, c2 = conv.weight.shape[0], conv.weight.shape[1]
        if bn.weight is None:
            raise NotImplementedError("dgx EdgeConv expects affine BatchNorm (as the reference builds it)")
        layers.append(_Layer(c2 // 2, co, bn, act.negative_slope))
        params += [conv.weight, bn.weight, bn.bias]
    return _EdgeConvStack.apply(x, k, layers, training, preps, *params)


def edgeconv_stack(x, k, convs, training):
    """Run the block chain. ``convs``: list of nn.Sequential(Conv2d(2C,Co,1,bias=False),
    BatchNorm2d(Co), LeakyReLU) exactly as the reference builds them (dgcnn.py:54-73).
    Returns the point-major concat buffer (B*N, sum Co)."""
    return edgeconv_stack_pair(x, k, convs, training)[0]
