"""Pointwise Conv(1x1) + BatchNorm + LeakyReLU on point-major features.

Replaces conv5 of reference models/dgcnn.py:74-78, 100-102: the reference
concatenates x1..x4 into (B,512,N,1) and runs Conv2d -> BatchNorm2d ->
LeakyReLU -> view(B,emb,N). Here the input is the EdgeConv chain's point-major
concat buffer (B*N, 512) as is; Z = X W^T is one engine GEMM (bf16 MFMA with
the BN statistics in its epilogue, or the fp32 MFMA GEMM in parity mode), BN
statistics / affine / LeakyReLU and the transpose to the reference's (B,emb,N)
layout are libdgx passes (pointconv.hip), issued by the C++ schedule
(csrc/dgx_torch.cpp). BN follows nn.BatchNorm rules per
module (dgx.bn: batch or running statistics by the BN's own flags, biased
batch var for normalisation, unbiased for running_var, momentum or cumulative
average).
"""
import torch

from . import _native as nat
from . import cpu
from . import bn as bn_
from . import precision as prec


class _PointConvBNLReLU(torch.autograd.Function):
    """One autograd node over the C++ schedule (libdgx_torch.so:
    dgx_host::pointconv_forward / pointconv_backward, shared with the eager
    DGCNN op and the torch.library ops)."""

    @staticmethod
    @prec.no_autocast
    def forward(ctx, X, X16, B, N, bn, slope, nt, tn, bf16, op_opts, weight, gamma, beta):
        from . import host
        host.load()
        t, f, i, g = bn_.op_args(bn)
        if X16 is None:
            X16 = torch.empty(0, dtype=torch.bfloat16, device=X.device)
        out, saved = torch.ops.dgx_host.pointconv_forward(X.float(), X16, B, N, weight, gamma, beta, t,
                                                          f + [float(slope)], i, g, bool(bf16), nt, tn, op_opts)
        ctx.meta = (B, N, float(slope), not bn_.mode(bn)[0], g, bool(bf16), op_opts)
        ctx.save_for_backward(weight, *saved)
        return out

    @staticmethod
    @prec.no_autocast
    def backward(ctx, dout):
        B, N, slope, ev, g, bf16, op_opts = ctx.meta
        weight, *saved = ctx.saved_tensors
        dX, dW, dg, db = torch.ops.dgx_host.pointconv_backward(dout, saved, weight, B, N, slope, ev, g, bf16, op_opts)
        return dX, None, None, None, None, None, None, None, None, None, dW, dg, db


def pointconv_bn_lrelu(X, B, N, seq, training=None, X16=None, wprep=None):
    """X (B*N, K) point-major -> (B, Co, N) = LeakyReLU(BN(Conv1x1(X))) with the
    modules of ``seq`` = nn.Sequential(Conv2d(K,Co,1,bias=False) or Conv1d,
    BatchNorm2d/1d, LeakyReLU) (reference dgcnn.py:74-78). ``X16``: optional bf16 twin of X
    (the GEMM operand in bf16). ``wprep``: optional bf16 (W, W^T) of the conv
    weight already made for this step (gemm.prep_weights). GEMM precision:
    ``precision.effective()`` at entry (bf16 mode or fp16/bf16 autocast ->
    bf16 MFMA). ``training`` is accepted for call compatibility only (dgx.bn:
    each BN module's own flags decide). A host tensor takes the CPU path (dgx.cpu)."""
    if cpu.is_cpu(X):
        return cpu.pointconv_bn_lrelu(X, B, N, seq, training)
    nat.require_device(X)
    conv, bn, act = seq[0], seq[1], seq[2]
    if conv.bias is not None or bn.weight is None:
        raise NotImplementedError("dgx pointconv expects Conv(bias=False) + affine BatchNorm")
    nt, tn = wprep if wprep is not None else (None, None)
    from .edgeconv import opts
    eff = prec.effective()
    return _PointConvBNLReLU.apply(X, X16, B, N, bn, act.negative_slope, nt, tn, eff == "bf16",
                                   opts(eff == "fp32_split"), conv.weight, bn.weight, bn.bias)
