"""Pointwise Conv(1x1) + BatchNorm + LeakyReLU on point-major features.

Replaces conv5 of reference models/dgcnn.py:74-78, 100-102: the reference
concatenates x1..x4 into (B,512,N,1) and runs Conv2d -> BatchNorm2d ->
LeakyReLU -> view(B,emb,N). Here the input is the EdgeConv chain's point-major
concat buffer (B*N, 512) as is; Z = X W^T is one engine GEMM (bf16 MFMA with
the BN statistics in its epilogue, or the fp32 MFMA GEMM in parity mode), BN
statistics / affine / LeakyReLU and the transpose to the reference's (B,emb,N)
layout are libdgx passes (pointconv.hip). BN follows nn.BatchNorm rules per
module (dgx.bn: batch or running statistics by the BN's own flags, biased
batch var for normalisation, unbiased for running_var, momentum or cumulative
average).
"""
import torch

from . import _native as nat
from . import cpu
from . import bn as bn_
from . import gemm as G
from . import precision as prec


class _PointConvBNLReLU(torch.autograd.Function):
    @staticmethod
    @prec.no_autocast
    def forward(ctx, X, X16, B, N, bn, slope, wprep_in, weight, gamma, beta):
        L = nat.lib()
        X = X.float()
        dev = X.device
        stream = nat.stream_of(X)
        M, K = X.shape
        Co = weight.shape[0]
        W = weight.reshape(Co, K)
        use_batch, _ = bn_.mode(bn)
        bf16 = prec.get() == "bf16"
        gemm_part = None
        wprep = None
        Xop = X
        z16 = False
        if bf16:  # bf16 MFMA GEMM (gemm.hip) with the BN column statistics fused in its epilogue
            if X16 is not None and X16.numel() and G.lds_ok_nt(X16, K):
                # bf16 twin of the concat buffer + bf16 W / W^T: LDS-DMA staged operands;
                # Z is stored bf16 (as autocast stores a conv output), stats from fp32 sums
                Xop = X16
                wprep = wprep_in if wprep_in is not None else G.prep_weight(weight, Co, K, False)
                with G.tag("conv5_fwd"):
                    if use_batch:
                        Z, gemm_part = G.lds_xwt(X16, wprep[0], stats=True, out_bf16=True)
                    else:
                        Z = G.lds_xwt(X16, wprep[0])
                z16 = Z.dtype == torch.bfloat16
            else:
                res = G.mm_xwt(X, W, stats=use_batch)
                Z, gemm_part = res if use_batch else (res, None)
        else:
            Z = prec.mm(X, W.t())  # (M, Co) fp32
        out = torch.empty((B, Co, N), dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            if use_batch:
                if gemm_part is not None:
                    partials, rows = gemm_part, gemm_part.shape[0]
                else:
                    rows = L.dgx_colstats_rows(M)
                    partials = torch.empty((rows, 2, Co), dtype=torch.float32, device=dev)
                    nat.check(L.dgx_colstats_f32(nat.f32(Z), Co, M, Co, nat.f32(partials), rows, stream), "colstats")
                st = bn_.batch_stats(partials, rows, float(M), bn, gamma, beta, stream)
            else:
                st = bn_.running_stats(bn, gamma, beta, stream)
            if z16:
                nat.check(L.dgx_pointconv_apply_bf16(nat.bf16(Z), B, N, Co, nat.f32(st.scale), nat.f32(st.shift),
                                                     float(slope), nat.f32(out), stream), "pointconv apply bf16")
            else:
                nat.check(L.dgx_pointconv_apply_f32(nat.f32(Z), Co, B, N, Co, nat.f32(st.scale), nat.f32(st.shift),
                                                    float(slope), nat.f32(out), stream), "pointconv apply")
        ctx.meta = (B, N, float(slope), bf16)
        ctx.st = st
        ctx.wprep = wprep
        ctx.wshape = weight.shape
        ctx.save_for_backward(Xop, W, Z)
        return out

    @staticmethod
    @prec.no_autocast
    def backward(ctx, dout):
        Xop, W, Z = ctx.saved_tensors
        st = ctx.st
        B, N, slope, bf16 = ctx.meta
        L = nat.lib()
        dev = Z.device
        stream = nat.stream_of(Z)
        M, Co = Z.shape
        dout = dout.float().contiguous()
        z16 = Z.dtype == torch.bfloat16
        rows = L.dgx_pointconv_bf16_rows(B, N) if z16 else L.dgx_pointconv_bwd_rows(B, N)
        partials = torch.empty((rows, 2, Co), dtype=torch.float32, device=dev)
        dZ = torch.empty((M, Co), dtype=torch.bfloat16 if bf16 else torch.float32, device=dev)
        sc, sh, mu, ist = nat.f32(st.scale), nat.f32(st.shift), nat.f32(st.mean), nat.f32(st.invstd)
        with torch.cuda.device(dev):
            if z16:  # two passes over (dout, Z): BN-backward reductions, then dZ directly
                nat.check(L.dgx_pointconv_bwd_bf16(nat.f32(dout), nat.bf16(Z), B, N, Co, sc, sh, mu, ist, slope, None,
                                                   None, nat.f32(partials), None, 0, stream), "pointconv bwd stats")
            else:
                dz = torch.empty((M, Co), dtype=torch.float32, device=dev)
                nat.check(L.dgx_pointconv_bwd_f32(nat.f32(dout), nat.f32(Z), Co, B, N, Co, sc, sh, mu, ist, slope,
                                                  nat.f32(dz), nat.f32(partials), stream), "pointconv bwd")
            dgamma, dbeta, c0, c1 = bn_.backward_consts(partials, rows, float(M), st, stream)
            if z16:
                nat.check(L.dgx_pointconv_bwd_bf16(nat.f32(dout), nat.bf16(Z), B, N, Co, sc, sh, None, None, slope,
                                                   nat.f32(c0), nat.f32(c1), None, nat.bf16(dZ), 1, stream),
                          "pointconv bwd dZ")
            else:
                nat.check(L.dgx_pointconv_input_grad(nat.f32(dz), nat.f32(Z), Co, M, Co, sc, nat.f32(c0), nat.f32(c1),
                                                     nat.ptr(dZ, nat.F32, nat.BF16), int(bf16), stream),
                          "pointconv dZ")
        if bf16:  # bf16 MFMA: dW = dZ^T X (split-K, deterministic), dX = dZ W
            dW = torch.empty((Co, Xop.shape[1]), dtype=torch.float32, device=dev)
            if ctx.wprep is not None:
                with G.tag("conv5_dW"):
                    G.lds_atb(dZ, Xop, dW)
                with G.tag("conv5_dX"):
                    dX = G.lds_xwt(dZ, ctx.wprep[1])
            else:
                G.mm_atb(dZ, Xop, dW)
                dX = G.mm_xw(dZ, W)
        else:   # fp32 MFMA GEMMs (dW: split-K over the B*N rows)
            dW = prec.mm(dZ.t(), Xop)
            dX = prec.mm(dZ, W)
        return dX, None, None, None, None, None, None, dW.view(ctx.wshape), dgamma, dbeta


def pointconv_bn_lrelu(X, B, N, seq, training=None, X16=None, wprep=None):
    """X (B*N, K) point-major -> (B, Co, N) = LeakyReLU(BN(Conv1x1(X))) with the
    modules of ``seq`` = nn.Sequential(Conv2d(K,Co,1,bias=False) or Conv1d,
    BatchNorm2d/1d, LeakyReLU) (reference dgcnn.py:74-78). ``X16``: optional bf16 twin of X
    (precision "bf16"), the GEMM operand. ``wprep``: optional bf16 (W, W^T) of
    the conv weight already made for this step (gemm.prep_weights).
    ``training`` is accepted for call compatibility only (dgx.bn: each BN
    module's own flags decide). A host tensor takes the CPU path (dgx.cpu)."""
    if cpu.is_cpu(X):
        return cpu.pointconv_bn_lrelu(X, B, N, seq, training)
    nat.require_device(X)
    conv, bn, act = seq[0], seq[1], seq[2]
    if conv.bias is not None or bn.weight is None:
        raise NotImplementedError("dgx pointconv expects Conv(bias=False) + affine BatchNorm")
    return _PointConvBNLReLU.apply(X, X16, B, N, bn, act.negative_slope, wprep, conv.weight, bn.weight, bn.bias)
