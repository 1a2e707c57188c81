"""Pointwise Conv(1x1) + BatchNorm + LeakyReLU on point-major features.

Replaces conv5 of reference models/dgcnn.py:74-78, 100-102: the reference
concatenates x1..x4 into (B,512,N,1) and runs Conv2d -> BatchNorm2d ->
LeakyReLU -> view(B,emb,N). Here the input is the EdgeConv chain's point-major
concat buffer (B*N, 512) as is; Z = X W^T is one GEMM (precision.mm), BN
statistics / affine / LeakyReLU and the transpose to the reference's (B,emb,N)
layout are libdgx passes (pointconv.hip). BN follows nn.BatchNorm rules
(biased batch var for normalisation, unbiased for running_var, momentum or
cumulative average).
"""
import torch

from . import _native as nat
from . import dist as dist_
from . import gemm as G
from . import precision as prec
from .edgeconv import _bn_factor


class _PointConvBNLReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, X16, B, N, bn, slope, training, wprep_in, weight, gamma, beta):
        L = nat.lib()
        dev = X.device
        stream = nat.stream_of(X)
        M, K = X.shape
        Co = weight.shape[0]
        W = weight.reshape(Co, K)
        use_batch = training or bn.running_mean is None
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
                    Z, gemm_part = G.lds_xwt(X16, wprep[0], stats=True, out_bf16=True)
                z16 = True
            else:
                res = G.mm_xwt(X, W, stats=use_batch)
                Z, gemm_part = res if use_batch else (res, None)
        else:
            Z = prec.mm(X, W.t())  # (M, Co) fp32
        scale = torch.empty(Co, dtype=torch.float32, device=dev)
        shift = torch.empty_like(scale)
        mean = torch.empty_like(scale)
        invstd = torch.empty_like(scale)
        out = torch.empty((B, Co, N), dtype=torch.float32, device=dev)
        sync, group = False, None
        with torch.cuda.device(dev):
            if use_batch:
                if gemm_part is not None:
                    partials, rows = gemm_part, gemm_part.shape[0]
                else:
                    rows = L.dgx_colstats_rows(M)
                    partials = torch.empty((rows, 2, Co), dtype=torch.float32, device=dev)
                    nat.check(L.dgx_colstats_f32(nat.ptr(Z), Co, M, Co, nat.ptr(partials), rows, stream),
                              "colstats")
                update = training and bn.running_mean is not None
                factor, nbt = _bn_factor(bn) if update else (0.0, None)
                fcount = float(M)
                sync, group = dist_.sync_group(bn, training)
                if sync:  # SyncBatchNorm: statistics of the global batch, one all-reduce
                    tot, fcount = dist_.allreduce_sums(partials.sum(0), fcount, group)
                    partials, rows = tot.unsqueeze(0).contiguous(), 1
                nat.check(L.dgx_bn_finalize_f32(
                    nat.ptr(partials), rows, Co, fcount, nat.ptr(gamma), nat.ptr(beta),
                    nat.ptr(bn.running_mean) if update else None, nat.ptr(bn.running_var) if update else None,
                    factor, float(bn.eps), nat.ptr(scale), nat.ptr(shift), nat.ptr(mean), nat.ptr(invstd),
                    nat.ptr(nbt), stream), "bn finalize")
            else:
                nat.check(L.dgx_bn_eval_affine_f32(
                    Co, nat.ptr(gamma), nat.ptr(beta), nat.ptr(bn.running_mean), nat.ptr(bn.running_var),
                    float(bn.eps), nat.ptr(scale), nat.ptr(shift), stream), "bn eval affine")
                # z-hat of the running statistics, for dgamma if eval-mode output is differentiated
                mean.copy_(bn.running_mean)
                invstd.copy_(torch.rsqrt(bn.running_var + bn.eps))
            if z16:
                nat.check(L.dgx_pointconv_apply_bf16(nat.ptr(Z), B, N, Co, nat.ptr(scale), nat.ptr(shift),
                                                     float(slope), nat.ptr(out), stream), "pointconv apply bf16")
            else:
                nat.check(L.dgx_pointconv_apply_f32(nat.ptr(Z), Co, B, N, Co, nat.ptr(scale), nat.ptr(shift),
                                                    float(slope), nat.ptr(out), stream), "pointconv apply")
        ctx.meta = (B, N, float(slope), use_batch, bf16)
        ctx.group = group if (use_batch and sync) else None
        ctx.wprep = wprep
        ctx.save_for_backward(Xop, W, Z, scale, shift, mean, invstd)
        return out

    @staticmethod
    def backward(ctx, dout):
        Xop, W, Z, scale, shift, mean, invstd = ctx.saved_tensors
        B, N, slope, use_batch, bf16 = ctx.meta
        L = nat.lib()
        dev = Z.device
        stream = nat.stream_of(Z)
        M, Co = Z.shape
        dout = dout.contiguous()
        z16 = Z.dtype == torch.bfloat16
        rows = L.dgx_pointconv_bf16_rows(B, N) if z16 else L.dgx_pointconv_bwd_rows(B, N)
        partials = torch.empty((rows, 2, Co), dtype=torch.float32, device=dev)
        dgamma = torch.empty(Co, dtype=torch.float32, device=dev)
        dbeta = torch.empty_like(dgamma)
        c0 = torch.empty_like(dgamma)
        c1 = torch.empty_like(dgamma)
        dZ = torch.empty((M, Co), dtype=torch.bfloat16 if bf16 else torch.float32, device=dev)
        with torch.cuda.device(dev):
            if z16:  # two passes over (dout, Z): BN-backward reductions, then dZ directly
                nat.check(L.dgx_pointconv_bwd_bf16(nat.ptr(dout), nat.ptr(Z), B, N, Co, nat.ptr(scale),
                                                   nat.ptr(shift), nat.ptr(mean), nat.ptr(invstd), slope, None, None,
                                                   nat.ptr(partials), None, 0, stream), "pointconv bwd stats")
            else:
                dz = torch.empty((M, Co), dtype=torch.float32, device=dev)
                nat.check(L.dgx_pointconv_bwd_f32(nat.ptr(dout), nat.ptr(Z), Co, B, N, Co, nat.ptr(scale),
                                                  nat.ptr(shift), nat.ptr(mean), nat.ptr(invstd), slope, nat.ptr(dz),
                                                  nat.ptr(partials), stream), "pointconv bwd")
            if use_batch and ctx.group is not None:  # SyncBatchNorm (see dgx.dist)
                loc = partials.sum(0)
                tot, gcount = dist_.allreduce_sums(loc, float(M), ctx.group)
                tot = tot.unsqueeze(0).contiguous()
                nat.check(L.dgx_bn_bwd_finalize_f32(nat.ptr(tot), 1, Co, gcount, nat.ptr(scale), nat.ptr(mean),
                                                    nat.ptr(invstd), None, None, nat.ptr(c0), nat.ptr(c1), 0,
                                                    stream), "bn bwd finalize")
                dbeta.copy_(loc[0])
                dgamma.copy_(loc[1])
            elif use_batch:
                nat.check(L.dgx_bn_bwd_finalize_f32(nat.ptr(partials), rows, Co, float(M), nat.ptr(scale),
                                                    nat.ptr(mean), nat.ptr(invstd), nat.ptr(dgamma), nat.ptr(dbeta),
                                                    nat.ptr(c0), nat.ptr(c1), 0, stream), "bn bwd finalize")
            else:  # running-stats BN: affine only
                c0.zero_()
                c1.zero_()
                sums = partials.sum(0)
                dbeta.copy_(sums[0])
                dgamma.copy_(sums[1])
            if z16:
                nat.check(L.dgx_pointconv_bwd_bf16(nat.ptr(dout), nat.ptr(Z), B, N, Co, nat.ptr(scale),
                                                   nat.ptr(shift), None, None, slope, nat.ptr(c0), nat.ptr(c1), None,
                                                   nat.ptr(dZ), 1, stream), "pointconv bwd dZ")
            else:
                nat.check(L.dgx_pointconv_input_grad(nat.ptr(dz), nat.ptr(Z), Co, M, Co, nat.ptr(scale),
                                                     nat.ptr(c0), nat.ptr(c1), nat.ptr(dZ), int(bf16), stream),
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
        else:
            dW = torch.mm(dZ.t(), Xop)
            dX = torch.mm(dZ, W)
        return dX, None, None, None, None, None, None, None, dW.view(Co, -1, 1, 1), dgamma, dbeta


def pointconv_bn_lrelu(X, B, N, seq, training, X16=None, wprep=None):
    """X (B*N, K) point-major -> (B, Co, N) = LeakyReLU(BN(Conv1x1(X))) with the
    modules of ``seq`` = nn.Sequential(Conv2d(K,Co,1,bias=False), BatchNorm2d,
    LeakyReLU) (reference dgcnn.py:74-78). ``X16``: optional bf16 twin of X
    (precision "bf16"), the GEMM operand. ``wprep``: optional bf16 (W, W^T) of
    the conv weight already made for this step (gemm.prep_weights)."""
    nat.require_device(X)
    conv, bn, act = seq[0], seq[1], seq[2]
    if conv.bias is not None or bn.weight is None:
        raise NotImplementedError("dgx pointconv expects Conv(bias=False) + affine BatchNorm")
    return _PointConvBNLReLU.apply(X, X16, B, N, bn, act.negative_slope, training, wprep, conv.weight, bn.weight,
                                   bn.bias)
