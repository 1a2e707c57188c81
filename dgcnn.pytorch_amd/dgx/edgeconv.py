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

BatchNorm decisions follow each BN module's own flags (dgx.bn). Under
torch.autocast the op runs in the engine's own precision on fp32 inputs
(precision.no_autocast): its GEMMs never return autocast-reduced products.
"""
import ctypes
import os
import threading

import torch

from . import _native as nat
from . import bn as bn_
from . import cpu
from . import gemm as G
from . import precision as prec
from .ops import knn_image_buffers, knn_raw, reduction_order

_tls = threading.local()

# bf16 mode: the backward scatter reads packed dz|slot words (DGX_SCATTER_PACKED=0:
# separate dz and slot arrays, A/B only; cfg2 step 1.4178 -> 1.4131 ms)
SCATTER_PACKED = os.environ.get("DGX_SCATTER_PACKED", "1") == "1"
# BN backward finalize folded into the scatter's prologue (DGX_FOLD_BN_BWD=0: a
# separate finalize launch, A/B only; cfg2 step 1.4131 -> 1.4065 ms)
FOLD_BN_BWD = os.environ.get("DGX_FOLD_BN_BWD", "1") == "1"
# blocks 1-3: the BN + LeakyReLU apply also writes the next block's kNN operand
# image and |x|^2 (dgx_bn_lrelu_apply_knn_image_f32), so that kNN skips its
# prepare pass (DGX_FUSE_KNN_IMAGE=0: separate prepare pass, A/B only)
FUSE_KNN_IMAGE = os.environ.get("DGX_FUSE_KNN_IMAGE", "1") == "1"
# bf16 backward: block l's input-gradient GEMM applies block l-1's LeakyReLU'
# in its epilogue and writes that block's packed dz + BN partials
# (dgx_gemm_edge_dz_bf16) instead of dY (DGX_FUSE_EDGE_DZ=0: dY + a dz pass)
FUSE_EDGE_DZ = os.environ.get("DGX_FUSE_EDGE_DZ", "1") == "1"


def debug_capture():
    """Per-thread capture dict for tests/tools (None when off): forward stores each
    block's routing decisions (idx, arg, zpos) under ("fwd", l), backward stores
    intermediates under l."""
    return getattr(_tls, "debug", None)


def set_debug_capture(d):
    _tls.debug = d


def _reverse_graphs(idxs, B, N, k, dev):
    """Reverse kNN graphs (CSR of in-edges) of all blocks in one launch
    (dgx_graph_reverse_multi), on the current stream at the start of the
    backward: the blocks' workgroups share the chip, and each cloud's index
    list is re-scanned by fewer workgroups than per-block launches need. (A
    build on a side stream overlapping the forward measured slower: 1.63 vs
    1.56 ms/step at cfg2, the concurrent kernels contend for the L2 the kNN
    operand images live in.)"""
    M = B * N
    n = len(idxs)
    rowptrs = [torch.empty(M + 1, dtype=torch.int32, device=dev) for _ in range(n)]
    edges = [torch.empty(M * k, dtype=torch.int32, device=dev) for _ in range(n)]
    arr = ctypes.c_void_p * n
    with torch.cuda.device(dev):
        nat.check(nat.lib().dgx_graph_reverse_multi(
            n, arr(*[i.data_ptr() for i in idxs]), B, N, k, arr(*[r.data_ptr() for r in rowptrs]),
            arr(*[e.data_ptr() for e in edges]), nat.stream_of(idxs[0])), "reverse graphs")
    return list(zip(rowptrs, edges))


class _Layer:
    """Non-tensor description of one block (weights are passed as tensors)."""

    def __init__(self, cin, cout, bn, slope):
        self.cin, self.cout, self.bn, self.slope = cin, cout, bn, slope


def split_weight(w, cin, cout):
    """Reference conv weight (Co, 2C[,1,1]) = [W1 | W2] -> stacked [W1; W2] (2Co, C):
    rows [0,Co) produce P (neighbour half, channels [0,C)), rows [Co,2Co) Q (centre half)."""
    w = w.reshape(cout, 2 * cin)
    return torch.cat([w[:, :cin], w[:, cin:]], dim=0)


def edge_select(PQ, idx, B, N, k, co, gamma, stream):
    """dgx_edge_fwd_gather_f32: per (point, channel) the selected pre-BN value,
    its slot, sum_k P_j and the per-block BN partial sums over all edges."""
    L = nat.lib()
    dev = PQ.device
    M = B * N
    ysel = torch.empty((M, co), dtype=torch.float32, device=dev)
    arg = torch.empty((M, co), dtype=torch.uint8, device=dev)
    sumP = torch.empty((M, co), dtype=torch.float32, device=dev)
    prow = L.dgx_edge_partials_rows(B, N, co)
    partials = torch.empty((prow, 2, co), dtype=torch.float32, device=dev)
    nat.check(L.dgx_edge_fwd_gather_f32(nat.f32(PQ), PQ.stride(0), nat.i32(idx), B, N, k, co, nat.f32(gamma),
                                        nat.f32(ysel), nat.u8(arg), nat.f32(sumP), nat.f32(partials), prow, stream),
              "edge gather")
    return ysel, arg, sumP, partials, prow


class _EdgeConvStack(torch.autograd.Function):
    @staticmethod
    @prec.no_autocast
    def forward(ctx, x, k, layers, ctx_preps, need_grad, *params):
        x = x.float()
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
        x_pm = x.permute(0, 2, 1).reshape(M, C0).contiguous()  # point-major rows (B = 1 reshapes to a view)
        saved = []
        off_in = None
        count = float(M * k)
        have16 = False  # xcat16 holds the previous block's output
        # bf16 [W1;W2] and transposed copies of blocks 2.. in one launch (used when
        # the block's input is the bf16 twin, i.e. after a selecting block)
        preps = list(ctx_preps) if ctx_preps is not None else [None] * len(layers)
        if bf16 and len(layers) > 1 and ctx_preps is None:
            jobs = [(params[3 * li], ly.cout, ly.cin, True, True) for li, ly in enumerate(layers) if li > 0]
            preps[1:] = G.prep_weights(jobs)
        dbg = debug_capture()
        next_prepared = None   # the next block's kNN image, written by this block's apply
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
                              strides=(N * total, 1, total), shape=(B, cin, N), prepared=next_prepared)
            next_prepared = None
            wprep = None
            if cin <= G.SMALLK_MAX:
                # raw coordinates (block 1, K = 3): exact fp32 in every mode
                PQ = G.mm_smallk_split(X, w, co)
            elif bf16:
                X16 = xcat16[:, off_in:off_in + cin] if li > 0 else None
                if have16 and G.lds_ok_nt(X16, cin):
                    # bf16 operands by LDS-DMA; the weight's bf16 [W1;W2] and transpose serve fwd and bwd
                    wprep = preps[li]
                    PQ = G.lds_xwt(X16, wprep[0])
                else:
                    PQ = G.mm_xwt(X, split_weight(w, cin, co))  # fp32 operands rounded while staged
            else:
                PQ = prec.mm(X, split_weight(w, cin, co).t())
            off = sum(widths[:li])
            out = xcat[:, off:off + co]
            bn = ly.bn
            use_batch, _ = bn_.mode(bn)
            with torch.cuda.device(dev):
                if use_batch or need_grad:
                    ysel, arg, sumP, partials, prow = edge_select(PQ, idx, B, N, k, co, gamma, stream)
                    if use_batch:
                        st = bn_.batch_stats(partials, prow, count, bn, gamma, beta, stream)
                    else:  # running statistics, output differentiated: keep the selection
                        st = bn_.running_stats(bn, gamma, beta, stream)
                if use_batch or need_grad:
                    out16 = xcat16[:, off:off + co] if bf16 else None
                    if FUSE_KNN_IMAGE and li + 1 < len(layers) and co in (64, 128) and N % 32 == 0:
                        next_prepared = knn_image_buffers(B, co, N, dev)
                        nat.check(L.dgx_bn_lrelu_apply_knn_image_f32(
                            nat.f32(ysel), B, N, co, nat.f32(st.scale), nat.f32(st.shift), float(ly.slope),
                            nat.f32(out), total, nat.ptr(out16, nat.BF16), nat.f32(next_prepared[0]),
                            nat.f32(next_prepared[1]), next_prepared[1].numel() * 4, stream), "bn apply + knn image")
                    else:
                        nat.check(L.dgx_bn_lrelu_apply_f32(nat.f32(ysel), M, co, nat.f32(st.scale),
                                                           nat.f32(st.shift), float(ly.slope), nat.f32(out), total,
                                                           nat.ptr(out16, nat.BF16), stream), "bn apply")
                    have16 = bf16
                    saved.append((idx, PQ, ysel, arg, sumP, st, wprep))
                    if dbg is not None:
                        # sign of fmaf(scale, ysel, shift) as the kernels evaluate it: the fp64
                        # product of two fp32 values is exact, so this sign is fma's sign
                        zpos = (st.scale.double() * ysel.double() + st.shift.double()) > 0
                        dbg[("fwd", li)] = (idx.clone(), arg.clone(), zpos)
                else:  # inference with running statistics: one fused select + affine + LReLU pass
                    st = bn_.running_stats(bn, gamma, beta, stream)
                    nat.check(L.dgx_edge_fwd_eval_f32(
                        nat.f32(PQ), PQ.stride(0), nat.i32(idx), B, N, k, co, nat.f32(st.scale), nat.f32(st.shift),
                        float(ly.slope), nat.f32(out), total, stream), "edge eval")
                    have16 = False
                    saved.append(None)
            off_in = off
        if dbg is not None:
            # the blocks' own inputs (tests re-derive each block's kNN and decisions from them)
            dbg["xcat"] = xcat
            dbg["xcat16"] = xcat16 if have16 else None
        ctx.k = k
        ctx.layers = layers
        ctx.shape = (B, C0, N)
        ctx.layer_state = saved
        ctx.x_needs_grad = ctx.needs_input_grad[0]
        ctx.bf16 = bf16
        ctx.save_for_backward(x_pm, xcat, xcat16, *params)
        if xcat16 is None or not have16:
            xcat16 = torch.empty(0, dtype=torch.bfloat16, device=dev)
        ctx.mark_non_differentiable(xcat16)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the bf16 twin
        return xcat, xcat16

    @staticmethod
    @prec.no_autocast
    def backward(ctx, dxcat, _unused):
        if dxcat is None:
            return (None,) * (5 + len(ctx.saved_tensors) - 3)
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
        dbg = debug_capture()
        if dxcat.dtype != torch.float32:
            dxcat = dxcat.float()
        if bf16:
            # The incoming gradient stays read-only: block l's input gradient is written
            # as addend (incoming slice) + dPQ Wcat into a fresh buffer, no clone pass.
            dxcat = dxcat.contiguous()
            lead = total - widths[-1]
            dnew = torch.empty((M, max(lead, 1)), dtype=torch.float32, device=dev)
        else:
            dxcat = dxcat.contiguous().clone()
        for idx in (st[0] for st in ctx.layer_state):
            assert idx.dtype == torch.int32 and idx.is_contiguous()
        rev = _reverse_graphs([st[0] for st in ctx.layer_state], B, N, k, dev)
        fused_dz = {}   # block -> (packed dz, partials, rows) made by the next block's dX GEMM
        for li in reversed(range(nl)):
            ly = layers[li]
            cin, co = ly.cin, ly.cout
            w = params[3 * li]
            idx, PQ, ysel, arg, sumP, st, wprep = ctx.layer_state[li]
            rowptr, edges = rev[li]
            off = sum(widths[:li])
            prev = off - widths[li - 1] if li > 0 else None
            X = x_pm if li == 0 else xcat[:, prev: prev + cin]
            if bf16 and li < nl - 1:
                dY, ldy = dnew[:, off:off + co], dnew.stride(0)
            else:
                dY, ldy = dxcat[:, off:off + co], dxcat.stride(0)
            pre = fused_dz.pop(li, None)
            if pre is not None:   # dz + partials already made by block li+1's dX GEMM epilogue
                dz, partials, nblk = pre
                dY = None
            else:
                nblk = max(1, min(1024, (M + 63) // 64))
                dz = torch.empty((M, co), dtype=torch.float32, device=dev)  # dL/dz at the selected edge
                partials = torch.empty((nblk, 2, co), dtype=torch.float32, device=dev)
            # dPQ only feeds the GEMMs: bf16 (what the GEMM would round it to) in bf16 mode
            dPQ = torch.empty((M, 2 * co), dtype=torch.bfloat16 if bf16 else torch.float32, device=dev)
            with torch.cuda.device(dev):
                bn_args = (M, co, nat.f32(st.scale), nat.f32(st.shift), nat.f32(st.mean), nat.f32(st.invstd),
                           float(ly.slope), nat.f32(dz), nat.f32(partials), nblk, stream)
                packed = bf16 and SCATTER_PACKED
                if pre is not None:
                    pass
                elif packed:
                    # dz words carry the selected slot in their 6 low mantissa bits (the
                    # dPQ they feed is rounded to bf16): one LDS word per in-edge-channel
                    nat.check(L.dgx_edge_bwd_dz_packed_f32(nat.f32(dY), ldy, nat.f32(ysel), nat.u8(arg), *bn_args),
                              "edge bwd dz")
                else:
                    nat.check(L.dgx_edge_bwd_dz_f32(nat.f32(dY), ldy, nat.f32(ysel), *bn_args), "edge bwd dz")
                fold = st.group is None and FOLD_BN_BWD
                if fold:
                    # BN backward finalize in the scatter's prologue (one launch)
                    dgamma, dbeta, c0, c1 = (torch.empty(co, dtype=torch.float32, device=dev) for _ in range(4))
                    nat.check(L.dgx_edge_bwd_scatter_fin_f32(
                        nat.f32(PQ), PQ.stride(0), nat.i32(rowptr), nat.i32(edges), nat.f32(dz),
                        None if packed else nat.u8(arg), nat.f32(sumP), B, N, k, co, nat.f32(partials), nblk,
                        count, nat.f32(st.scale), nat.f32(st.mean), nat.f32(st.invstd), int(st.eval),
                        nat.f32(dgamma), nat.f32(dbeta), nat.f32(c0), nat.f32(c1), nat.ptr(dPQ, nat.F32, nat.BF16),
                        int(bf16), int(packed), stream), "edge bwd scatter")
                else:   # SyncBatchNorm: the all-reduce sits between the partials and the finalize
                    dgamma, dbeta, c0, c1 = bn_.backward_consts(partials, nblk, count, st, stream)
                common = (B, N, k, co, nat.f32(st.scale), nat.f32(c0), nat.f32(c1), nat.ptr(dPQ, nat.F32, nat.BF16),
                          int(bf16), stream)
                if not fold and packed:
                    nat.check(L.dgx_edge_bwd_scatter_packed_f32(
                        nat.f32(PQ), PQ.stride(0), nat.i32(rowptr), nat.i32(edges), nat.f32(dz), nat.f32(sumP),
                        *common), "edge bwd scatter")
                elif not fold:
                    nat.check(L.dgx_edge_bwd_scatter_f32(
                        nat.f32(PQ), PQ.stride(0), nat.i32(rowptr), nat.i32(edges), nat.f32(dz), nat.u8(arg),
                        nat.f32(sumP), *common), "edge bwd scatter")
            if dbg is not None:
                dbg[li] = {"dY": dY.clone() if dY is not None else None, "dz": dz.clone(), "dgamma": dgamma.clone(), "dbeta": dbeta.clone(),
                           "c0": c0.clone(), "c1": c1.clone(), "dPQ": dPQ.float(), "partials": partials.clone(),
                           "ysel": ysel.clone(), "scale": st.scale.clone(), "shift": st.shift.clone(),
                           "arg": arg.clone(), "idx": idx.clone(), "PQ": PQ.clone(), "sumP": sumP.clone(),
                           "mean": st.mean.clone(), "invstd": st.invstd.clone(), "X": X.clone(),
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
                    prev_state = ctx.layer_state[li - 1]
                    if wprep is not None and FUSE_EDGE_DZ and packed and prev_state is not None and G.edge_dz_ok(dPQ, cin):
                        _, _, ysel_p, arg_p, _, st_p, _ = prev_state
                        fused_dz[li - 1] = G.lds_xwt_edge_dz(dPQ, wprep[1], add, ysel_p, arg_p, st_p,
                                                             layers[li - 1].slope)
                    elif wprep is not None:
                        G.lds_xwt(dPQ, wprep[1], out=dst, addend=add)
                    else:
                        dst.copy_(add)
                        G.mm_xw(dPQ, split_weight(w, cin, co), out=dst, accumulate=True)
                elif ctx.x_needs_grad:
                    dx_in = G.mm_xw(dPQ, split_weight(w, cin, co)).view(B, N, C0).permute(0, 2, 1)
            else:
                wcat = split_weight(w, cin, co)
                dwcat = prec.mm(dPQ.t(), X)  # (2Co, C)
                grads[3 * li] = torch.cat([dwcat[:co], dwcat[co:]], dim=1).reshape(w.shape)
                if li > 0:
                    prec.mm(dPQ, wcat, out=dxcat[:, prev:prev + cin], accumulate=True)
                elif ctx.x_needs_grad:
                    dx_in = prec.mm(dPQ, wcat).view(B, N, C0).permute(0, 2, 1)
        return (dx_in, None, None, None, None, *grads)


def _layers_and_params(convs, weights=None):
    layers, params = [], []
    for li, seq in enumerate(convs):
        conv, bn, act = seq[0], seq[1], seq[2]
        co, c2 = conv.weight.shape[0], conv.weight.shape[1]
        if conv.bias is not None or bn.weight is None:
            raise NotImplementedError("dgx EdgeConv expects Conv2d(bias=False) + affine BatchNorm "
                                      "(as the reference builds them, dgcnn.py:54-73)")
        layers.append(_Layer(c2 // 2, co, bn, act.negative_slope))
        params += [conv.weight if weights is None else weights[li], bn.weight, bn.bias]
    return layers, params


def edgeconv_stack_pair(x, k, convs, training=None, preps=None, weights=None):
    """As edgeconv_stack, also returning the bf16 twin of the concat buffer
    (empty unless precision "bf16" produced it): conv5's GEMM operand.
    ``preps``: optional per-block bf16 weight copies (gemm.prep_weights) made
    by the caller in one launch with other layers' (None for block 1).
    ``training`` is accepted for call compatibility only: every BatchNorm
    decides batch vs running statistics by its own flags, as nn.BatchNorm does.
    ``weights``: per-block conv weights used instead of the modules' (the
    re-parameterised weights of DGCNN's edge_mode "diff"). A host tensor takes
    the CPU path (dgx.cpu)."""
    if cpu.is_cpu(x):
        return cpu.edgeconv_stack_pair(x, k, convs, training, weights=weights)
    nat.require_device(x)
    if x.dtype != torch.float32:
        x = x.float()
    layers, params = _layers_and_params(convs, weights)
    # whether this forward will be differentiated (inside Function.forward grad
    # mode is always off, so it is decided here)
    need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
    return _EdgeConvStack.apply(x, k, layers, preps, need_grad, *params)


def edgeconv_stack(x, k, convs, training=None):
    """Run the block chain. ``convs``: list of nn.Sequential(Conv2d(2C,Co,1,bias=False),
    BatchNorm2d(Co), LeakyReLU) exactly as the reference builds them (dgcnn.py:54-73).
    Returns the point-major concat buffer (B*N, sum Co)."""
    return edgeconv_stack_pair(x, k, convs, training)[0]
