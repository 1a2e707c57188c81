"""Fused EdgeConv stack: the DGCNN block chain of reference models/dgcnn.py:84-100.

Reference, per block l (dgcnn.py:84-98):
    e = get_graph_feature(x_{l-1}, k)                     (B, 2C, N, k)
    x_l = max_k LeakyReLU(BN(Conv2d_1x1(e)))               (B, Co, N)
and then cat(x1..x4) (dgcnn.py:100).

Engine: one autograd node for the whole chain, whose schedule is the C++ one
(csrc/dgx_torch.cpp: dgx_host::chain_forward / chain_backward, shared with the
eager DGCNN op and the torch.library ops). Activations live point-major in
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
fp16/bf16 torch.autocast the chain's GEMMs take the bf16 path
(precision.effective); kNN, BN and the elementwise work stay fp32.
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
from . import ops as _ops
from .ops import knn_raw, reduction_order

_tls = threading.local()

# bf16 mode (and the fp32 mode with split-bf16 conv5 GEMMs, SPLIT32): the
# backward scatter reads packed dz|slot words (DGX_SCATTER_PACKED=0: separate dz
# and slot arrays, A/B only; cfg2 step 1.4178 -> 1.4131 ms)
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
# split-bf16 fp32 GEMMs (precision "fp32_split", or fp16 autocast: see
# dgx.precision): conv5's GEMMs as 3 passes of the bf16 MFMA on split operands
# (x = hi + lo, 16 significant bits each: hi.W_hi + hi.W_lo + lo.W_hi, ~2^-16
# relative per product, fp32 sums) instead of the f32 MFMA, which runs at 1/16
# of the bf16 rate. DGX_SPLIT32=1 forces it in the plain "fp32" mode too (A/B);
# the "fp32" default keeps exact products and exact dz.
SPLIT32 = os.environ.get("DGX_SPLIT32", "0") == "1"
# ... and (when split) the EdgeConv blocks' weight and input gradients too: the
# backward scatter writes dPQ as its split planes and dW / dX run as the same
# 3-pass GEMMs (DGX_SPLIT32_EDGE=0: those two on the f32 MFMA)
SPLIT32_EDGE = os.environ.get("DGX_SPLIT32_EDGE", "1") == "1"
# backward scatter in push form (dgx_edge_bwd_scatter_push_f32): each source's
# selected dz is added to its target in exact 64-bit fixed point (order-free,
# the exact sum rounded once), the in-edge loop reads only Q rows. Measured
# slower than the pull form (cfg2 step 1.32 -> 1.41 ms, r06u): the scatter is
# bound by its per-workgroup latency chain, which the push phases lengthen.
# DGX_SCATTER_PUSH=1 selects it.
SCATTER_PUSH = os.environ.get("DGX_SCATTER_PUSH", "0") == "1"


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


def opts(split=None):
    """The A/B switches above and gemm.SLAB_CAP_MB as the C++ schedule's
    ``opts`` word (csrc/dgx_torch.cpp ``decode``). ``split``: whether the op's
    fp32 GEMMs run as split bf16 — decided at the op's entry
    (``precision.split()``, which sees autocast); None = the global mode's."""
    if split is None:
        split = prec.get() == "fp32_split"
    split = bool(split or SPLIT32)
    cap = max(0, min(255, int(G.SLAB_CAP_MB)))
    return (int(SCATTER_PACKED) | 2 * int(FOLD_BN_BWD) | 4 * int(FUSE_KNN_IMAGE) | 8 * int(FUSE_EDGE_DZ)
            | 16 * int(split) | 32 * int(SCATTER_PUSH) | 64 * int(split and SPLIT32_EDGE) | (cap << 8))


PER_LAYER = 9   # saved per block: idx, PQ, ysel, arg, sumP, scale, shift, mean, invstd


def _bn_lists(layers):
    bn_t, bn_f, bn_i, groups, slopes = [], [], [], [], []
    for ly in layers:
        t, f, i, g = bn_.op_args(ly.bn)
        bn_t += t
        bn_f += f + [float(ly.slope)]
        bn_i += i
        groups.append(g)
        slopes.append(float(ly.slope))
    return bn_t, bn_f, bn_i, groups, slopes


def capture_decisions(dbg, saved, xcat, xcat16):
    """Debug capture of one chain forward from its saved state: per selecting
    block ("fwd", l) = (idx, max/min slot, LeakyReLU sign), plus the blocks'
    inputs (tests re-derive each block's kNN and decisions from them)."""
    n = (len(saved) - 1) // PER_LAYER
    for li in range(n):
        t = saved[1 + PER_LAYER * li: 1 + PER_LAYER * (li + 1)]
        if t[0].numel() == 0:
            continue
        idx, ysel, arg, scale, shift = t[0], t[2], t[3], t[5], t[6]
        # sign of fmaf(scale, ysel, shift) as the kernels evaluate it: the fp64
        # product of two fp32 values is exact, so this sign is fma's sign
        zpos = (scale.double() * ysel.double() + shift.double()) > 0
        dbg[("fwd", li)] = (idx.clone(), arg.clone(), zpos)
    dbg["xcat"] = xcat
    dbg["xcat16"] = xcat16 if xcat16.numel() else None


class _EdgeConvStack(torch.autograd.Function):
    """The chain as one autograd node over the C++ schedule (libdgx_torch.so:
    dgx_host::chain_forward / chain_backward — the same code the eager DGCNN
    op and the torch.library ops run)."""

    @staticmethod
    @prec.no_autocast
    def forward(ctx, x, k, layers, prep, idx0, bf16, op_opts, need_grad, *params):
        from . import host
        host.load()
        x = x.float()
        weights, gammas, betas = list(params[0::3]), list(params[1::3]), list(params[2::3])
        bn_t, bn_f, bn_i, groups, slopes = _bn_lists(layers)
        xcat, xcat16, saved, prep_out = torch.ops.dgx_host.chain_forward(
            x, k, weights, gammas, betas, bn_t, bn_f, bn_i, groups, slopes, bool(bf16), bool(need_grad), prep, idx0,
            op_opts)
        dbg = debug_capture()
        if dbg is not None:
            capture_decisions(dbg, saved, xcat, xcat16)
        ctx.meta = (k, tuple(x.shape), bool(bf16), [int(not bn_.mode(ly.bn)[0]) for ly in layers], groups, slopes,
                    len(saved), op_opts)
        # x itself is saved: its version counter guards the point-major rows (a view of x)
        ctx.save_for_backward(x, xcat, xcat16, prep_out, *saved, *weights)
        ctx.mark_non_differentiable(xcat16)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the bf16 twin
        return xcat, xcat16

    @staticmethod
    @prec.no_autocast
    def backward(ctx, dxcat, _unused):
        k, shape, bf16, evals, groups, slopes, ns, op_opts = ctx.meta
        n = len(slopes)
        if dxcat is None:
            return (None,) * (8 + 3 * n)
        t = ctx.saved_tensors
        xcat, xcat16, prep = t[1], t[2], t[3]
        saved, weights = list(t[4:4 + ns]), list(t[4 + ns:])
        dx, dws, dgs, dbs = torch.ops.dgx_host.chain_backward(
            dxcat, xcat, xcat16, saved, weights, prep if prep.numel() else None, list(shape), k, evals, groups, slopes,
            bf16, ctx.needs_input_grad[0], op_opts)
        grads = [g for trip in zip(dws, dgs, dbs) for g in trip]
        return (dx if dx.numel() else None, None, None, None, None, None, None, None, *grads)


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
    ``preps``: optional bf16 weight-copy buffer whose first entries are blocks
    2..n's (gemm.prep_layout order, split stacked weights), made by the caller
    in one launch with other layers'; None makes them here.
    ``training`` is accepted for call compatibility only: every BatchNorm
    decides batch vs running statistics by its own flags, as nn.BatchNorm does.
    ``weights``: per-block conv weights used instead of the modules' (the
    re-parameterised weights of DGCNN's edge_mode "diff"). A host tensor takes
    the CPU path (dgx.cpu). GEMM precision: ``precision.effective()`` at entry
    (bf16 mode or fp16/bf16 autocast -> bf16 MFMA)."""
    if cpu.is_cpu(x):
        return cpu.edgeconv_stack_pair(x, k, convs, training, weights=weights)
    nat.require_device(x)
    if x.dtype != torch.float32:
        x = x.float()
    layers, params = _layers_and_params(convs, weights)
    eff = prec.effective()
    bf16 = eff == "bf16"
    # whether this forward will be differentiated (inside Function.forward grad
    # mode is always off, so it is decided here)
    need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
    idx0 = None
    if getattr(_ops._tls, "cache", None) is not None:
        # inside a kNN-sharing scope (Net.forward): block 1's kNN is the scope's entry
        idx0 = knn_raw(x.detach(), k, order=reduction_order(x), out_dtype=torch.int32)
    if isinstance(preps, (list, tuple)):
        preps = None
    return _EdgeConvStack.apply(x, k, layers, preps, idx0, bf16, opts(eff == "fp32_split"), need_grad, *params)


def edgeconv_stack(x, k, convs, training=None):
    """Run the block chain. ``convs``: list of nn.Sequential(Conv2d(2C,Co,1,bias=False),
    BatchNorm2d(Co), LeakyReLU) exactly as the reference builds them (dgcnn.py:54-73).
    Returns the point-major concat buffer (B*N, sum Co)."""
    return edgeconv_stack_pair(x, k, convs, training)[0]
