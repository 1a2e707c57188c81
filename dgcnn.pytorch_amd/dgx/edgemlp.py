"""PositionEmbedding's per-edge MLP: reference models/layers.py:45-52.

Reference:
    e  = get_graph_feature(x, k)                      (B, 2C, N, k)   layers.py:45
    h1 = conv1(e)   Conv2d(2C,64) + BN2d + LeakyReLU   per edge        layers.py:17-18, 48
    t  = conv2(h1)  Conv2d(64,128) + BN2d + LeakyReLU  per edge        layers.py:19-20, 49
    t  = t.max(dim=-1)[0]                             (B, 128, N)     layers.py:52

Engine: one autograd node. The edge tensor e is never built: conv1 is
decomposed into PQ = X [W1;W2]^T (y_e = P_j + Q_i, as in the EdgeConv chain),
its BN statistics come from the EdgeConv gather kernel, and h1 is written once
per edge row (E = B*N*k rows, point-major) straight in the dtype conv2's GEMM
consumes. conv2 is one MFMA GEMM over the E edge rows (bf16 with the BN
statistics fused in its epilogue, or fp32 in the parity mode); the max over k
keeps the selected value and slot. Backward: BN2 on the selected edges, a dense
dZ2, the two conv2 GEMMs (dH1, dW2), LReLU/BN1 backward in place and a
deterministic gather over the kNN graph and its reverse for dP/dQ.
"""
import torch

from . import _native as nat
from . import dist as dist_
from . import gemm as G
from . import precision as prec
from .edgeconv import _bn_factor, _split_weight
from .ops import knn_raw, reduction_order


def _bn_forward(L, dev, stream, partials, rows, count, bn, gamma, beta, training):
    """Batch statistics -> (scale, shift, mean, invstd, sync group or None)."""
    co = gamma.shape[0]
    scale = torch.empty(co, dtype=torch.float32, device=dev)
    shift, mean, invstd = torch.empty_like(scale), torch.empty_like(scale), torch.empty_like(scale)
    update = training and bn.running_mean is not None
    factor, nbt = _bn_factor(bn) if update else (0.0, None)
    sync, group = dist_.sync_group(bn, training)
    fin, frows, fcount = partials, rows, count
    if sync:  # SyncBatchNorm: statistics of the global batch, one all-reduce
        tot, fcount = dist_.allreduce_sums(partials.sum(0), count, group)
        fin, frows = tot.unsqueeze(0).contiguous(), 1
    nat.check(L.dgx_bn_finalize_f32(
        nat.ptr(fin), frows, co, fcount, nat.ptr(gamma), nat.ptr(beta),
        nat.ptr(bn.running_mean) if update else None, nat.ptr(bn.running_var) if update else None,
        factor, float(bn.eps), nat.ptr(scale), nat.ptr(shift), nat.ptr(mean), nat.ptr(invstd), nat.ptr(nbt),
        stream), "bn finalize")
    return scale, shift, mean, invstd, (group if sync else None)


def _bn_eval(L, dev, stream, bn, gamma, beta):
    co = gamma.shape[0]
    scale = torch.empty(co, dtype=torch.float32, device=dev)
    shift = torch.empty_like(scale)
    nat.check(L.dgx_bn_eval_affine_f32(co, nat.ptr(gamma), nat.ptr(beta), nat.ptr(bn.running_mean),
                                       nat.ptr(bn.running_var), float(bn.eps), nat.ptr(scale), nat.ptr(shift),
                                       stream), "bn eval affine")
    return scale, shift


def _bn_backward(L, dev, stream, partials, rows, count, scale, mean, invstd, group):
    """(dgamma, dbeta, c0, c1) of BN's train-mode backward from (sum g, sum g*yhat) partials."""
    co = scale.shape[0]
    dgamma = torch.empty(co, dtype=torch.float32, device=dev)
    dbeta, c0, c1 = torch.empty_like(dgamma), torch.empty_like(dgamma), torch.empty_like(dgamma)
    if group is None:
        nat.check(L.dgx_bn_bwd_finalize_f32(nat.ptr(partials), rows, co, count, nat.ptr(scale), nat.ptr(mean),
                                            nat.ptr(invstd), nat.ptr(dgamma), nat.ptr(dbeta), nat.ptr(c0),
                                            nat.ptr(c1), 0, stream), "bn bwd finalize")
    else:  # SyncBatchNorm: input gradient from global sums, gamma/beta grads rank-local
        loc = partials.sum(0)
        tot, gcount = dist_.allreduce_sums(loc, count, group)
        tot = tot.unsqueeze(0).contiguous()
        nat.check(L.dgx_bn_bwd_finalize_f32(nat.ptr(tot), 1, co, gcount, nat.ptr(scale), nat.ptr(mean),
                                            nat.ptr(invstd), None, None, nat.ptr(c0), nat.ptr(c1), 0, stream),
                  "bn bwd finalize")
        dbeta.copy_(loc[0])
        dgamma.copy_(loc[1])
    return dgamma, dbeta, c0, c1


class _EdgeMLP2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, bn1, bn2, slope1, slope2, training, w1, g1, b1, w2, g2, b2):
        dev = x.device
        B, C, N = x.shape
        M, E = B * N, B * N * k
        C1, C2 = w1.shape[0], w2.shape[0]
        L = nat.lib()
        stream = nat.stream_of(x)
        bf16 = prec.get() == "bf16"
        X = x.permute(0, 2, 1).reshape(M, C)
        idx = knn_raw(x, k, order=reduction_order(x), out_dtype=torch.int32)      # layers.py:45 -> dgcnn.py:21
        w1s = _split_weight(w1, C, C1)
        PQ = G.mm_xwt(X, w1s) if bf16 else prec.mm(X, w1s.t())                   # (M, 2C1)
        W2 = w2.reshape(C2, C1)
        use1 = training or bn1.running_mean is None
        use2 = training or bn2.running_mean is None
        st1 = st2 = None
        sumP1 = None
        with torch.cuda.device(dev):
            # ---- conv1: BN1 statistics over all E edges, then h1 per edge row
            if use1:
                ysel1 = torch.empty((M, C1), dtype=torch.float32, device=dev)
                arg1 = torch.empty((M, C1), dtype=torch.uint8, device=dev)
                sumP1 = torch.empty((M, C1), dtype=torch.float32, device=dev)
                prow = L.dgx_edge_partials_rows(B, N, C1)
                part1 = torch.empty((prow, 2, C1), dtype=torch.float32, device=dev)
                nat.check(L.dgx_edge_fwd_gather_f32(nat.ptr(PQ), 2 * C1, nat.ptr(idx), B, N, k, C1, nat.ptr(g1),
                                                    nat.ptr(ysel1), nat.ptr(arg1), nat.ptr(sumP1), nat.ptr(part1),
                                                    prow, stream), "edge gather (bn1 stats)")
                del ysel1, arg1  # only the statistics and sum_k P_j (for dQ) are used
                st1 = _bn_forward(L, dev, stream, part1, prow, float(E), bn1, g1, b1, training)
                scale1, shift1 = st1[0], st1[1]
            else:
                scale1, shift1 = _bn_eval(L, dev, stream, bn1, g1, b1)
            h16 = bf16 and C1 % 64 == 0
            H1 = torch.empty((E, C1), dtype=torch.bfloat16 if h16 else torch.float32, device=dev)
            nat.check(L.dgx_edge_mlp_h1_f32(nat.ptr(PQ), 2 * C1, nat.ptr(idx), B, N, k, C1, nat.ptr(scale1),
                                            nat.ptr(shift1), float(slope1), nat.ptr(H1), int(h16), stream), "edge h1")
            # ---- conv2: one GEMM over the edge rows (+ BN2 column statistics)
            wprep = None
            part2 = None
            if h16:
                wprep = G.prep_weight(w2, C2, C1, False)
                if use2:
                    Z2, part2 = G.lds_xwt(H1, wprep[0], stats=True, out_bf16=True)
                else:
                    Z2 = G.lds_xwt(H1, wprep[0])
            elif bf16:
                res = G.mm_xwt(H1, W2, stats=use2)
                Z2, part2 = res if use2 else (res, None)
            else:
                Z2 = prec.mm(H1, W2.t())
                if use2:
                    rows = L.dgx_colstats_rows(E)
                    part2 = torch.empty((rows, 2, C2), dtype=torch.float32, device=dev)
                    nat.check(L.dgx_colstats_f32(nat.ptr(Z2), C2, E, C2, nat.ptr(part2), rows, stream), "colstats")
            z16 = Z2.dtype == torch.bfloat16
            if use2:
                st2 = _bn_forward(L, dev, stream, part2, part2.shape[0], float(E), bn2, g2, b2, training)
                scale2, shift2 = st2[0], st2[1]
            else:
                scale2, shift2 = _bn_eval(L, dev, stream, bn2, g2, b2)
            # ---- max over k (layers.py:52) of LReLU(BN2(z2)): select, then apply
            ysel = torch.empty((M, C2), dtype=torch.float32, device=dev)
            arg = torch.empty((M, C2), dtype=torch.uint8, device=dev)
            nat.check(L.dgx_edge_mlp_max_f32(nat.ptr(Z2), int(z16), B, N, k, C2, nat.ptr(scale2), nat.ptr(ysel),
                                             nat.ptr(arg), stream), "edge max")
            out = torch.empty((M, C2), dtype=torch.float32, device=dev)
            nat.check(L.dgx_bn_lrelu_apply_f32(nat.ptr(ysel), M, C2, nat.ptr(scale2), nat.ptr(shift2),
                                               float(slope2), nat.ptr(out), C2, None, stream), "bn apply")
        ctx.dims = (B, C, N, k, C1, C2)
        ctx.slopes = (float(slope1), float(slope2))
        ctx.st = (st1, st2)
        ctx.wprep = wprep
        ctx.bf16 = bf16
        ctx.save_for_backward(X, idx, PQ, sumP1, H1, Z2, ysel, arg, w1, w2)
        return out.view(B, N, C2).permute(0, 2, 1)

    @staticmethod
    def backward(ctx, dout):
        st1, st2 = ctx.st
        if st1 is None or st2 is None:
            raise RuntimeError("dgx edge MLP: backward through an eval-mode (running-stats) forward is not supported")
        X, idx, PQ, sumP1, H1, Z2, ysel, arg, w1, w2 = ctx.saved_tensors
        B, C, N, k, C1, C2 = ctx.dims
        slope1, slope2 = ctx.slopes
        M, E = B * N, B * N * k
        dev = X.device
        L = nat.lib()
        stream = nat.stream_of(X)
        scale1, shift1, mean1, invstd1, group1 = st1
        scale2, shift2, mean2, invstd2, group2 = st2
        z16 = Z2.dtype == torch.bfloat16
        dY = dout.permute(0, 2, 1).reshape(M, C2).contiguous()
        with torch.cuda.device(dev):
            # ---- BN2 + LReLU backward at the selected edges, then dense over all edges
            nblk = max(1, min(1024, (M + 63) // 64))
            dz = torch.empty((M, C2), dtype=torch.float32, device=dev)
            part = torch.empty((nblk, 2, C2), dtype=torch.float32, device=dev)
            nat.check(L.dgx_edge_bwd_dz_f32(nat.ptr(dY), C2, nat.ptr(ysel), nat.ptr(arg), M, C2, nat.ptr(scale2),
                                            nat.ptr(shift2), nat.ptr(mean2), nat.ptr(invstd2), slope2, nat.ptr(dz),
                                            nat.ptr(part), nblk, stream), "edge bwd dz")
            dg2, db2, c0, c1 = _bn_backward(L, dev, stream, part, nblk, float(E), scale2, mean2, invstd2, group2)
            dZ2 = torch.empty((E, C2), dtype=Z2.dtype, device=dev)
            nat.check(L.dgx_edge_mlp_dz_f32(nat.ptr(dz), nat.ptr(Z2), int(z16), B, N, k, C2, nat.ptr(scale2),
                                            nat.ptr(c0), nat.ptr(c1), nat.ptr(dZ2), stream), "edge dz2")
            # ---- conv2 GEMMs: dH1 = dZ2 W2, dW2 = dZ2^T H1
            gw2 = torch.empty((C2, C1), dtype=torch.float32, device=dev)
            if ctx.wprep is not None and z16:
                dH1 = G.lds_xwt(dZ2, ctx.wprep[1])
                G.lds_atb(dZ2, H1, gw2)
            else:
                W2 = w2.reshape(C2, C1)
                dH1 = prec.mm(dZ2.float(), W2)
                gw2 = prec.mm(dZ2.float().t(), H1.float())
            # ---- LReLU + BN1 backward (per edge), then dP / dQ over the graph
            rows = L.dgx_edge_mlp_h1_bwd_rows(B, N, k, C1)
            part1 = torch.empty((rows, 2, C1), dtype=torch.float32, device=dev)
            nat.check(L.dgx_edge_mlp_h1_bwd_f32(nat.ptr(dH1), nat.ptr(PQ), 2 * C1, nat.ptr(idx), B, N, k, C1,
                                                nat.ptr(scale1), nat.ptr(shift1), nat.ptr(mean1), nat.ptr(invstd1),
                                                slope1, nat.ptr(part1), rows, stream), "edge h1 bwd")
            dg1, db1, e0, e1 = _bn_backward(L, dev, stream, part1, rows, float(E), scale1, mean1, invstd1, group1)
            rowptr = torch.empty(M + 1, dtype=torch.int32, device=dev)
            edges = torch.empty(E, dtype=torch.int32, device=dev)
            nat.check(L.dgx_graph_reverse(nat.ptr(idx), B, N, k, nat.ptr(rowptr), nat.ptr(edges), stream),
                      "reverse graph")
            dPQ = torch.empty((M, 2 * C1), dtype=torch.float32, device=dev)
            nat.check(L.dgx_edge_mlp_scatter_f32(nat.ptr(dH1), nat.ptr(PQ), 2 * C1, nat.ptr(sumP1), nat.ptr(rowptr),
                                                 nat.ptr(edges), B, N, k, C1, nat.ptr(scale1), nat.ptr(e0),
                                                 nat.ptr(e1), nat.ptr(dPQ), stream), "edge h1 scatter")
        # ---- conv1 (K = C, tiny): dW1 = [dP^T X | dQ^T X], dX = dP W1a + dQ W1b
        dx = None
        if ctx.bf16:  # the engine's GEMMs (split-K over the M rows, un-stacked in the slab sum)
            gw1 = torch.empty((C1, 2 * C), dtype=torch.float32, device=dev)
            G.mm_atb(dPQ, X, gw1, split_rows=C1)
            gw1 = gw1.view(w1.shape)
            if ctx.needs_input_grad[0]:
                dx = G.mm_xw(dPQ, _split_weight(w1, C, C1)).view(B, N, C).permute(0, 2, 1)
        else:
            dwcat = prec.mm(dPQ.t(), X)  # (2C1, C)
            gw1 = torch.cat([dwcat[:C1], dwcat[C1:]], dim=1).reshape(w1.shape)
            if ctx.needs_input_grad[0]:
                dx = prec.mm(dPQ, _split_weight(w1, C, C1)).view(B, N, C).permute(0, 2, 1)
        return (dx, None, None, None, None, None, None, gw1, dg1, db1, gw2.view(w2.shape), dg2, db2)


def edge_mlp2(x, k, conv1, conv2, training):
    """max_k conv2(conv1(get_graph_feature(x, k))) for conv1/conv2 =
    nn.Sequential(Conv2d(1x1, bias=False), BatchNorm2d, LeakyReLU) as
    PositionEmbedding builds them (reference models/layers.py:17-20, 45-52).
    Returns (B, C2, N) (a permuted view of a point-major buffer)."""
    nat.require_device(x)
    if x.dtype != torch.float32:
        x = x.float()
    (cv1, bn1, act1), (cv2, bn2, act2) = (conv1[0], conv1[1], conv1[2]), (conv2[0], conv2[1], conv2[2])
    if bn1.weight is None or bn2.weight is None:
        raise NotImplementedError("dgx edge MLP expects affine BatchNorm (as the reference builds it)")
    c1w, c2w = cv1.weight.shape[0], cv2.weight.shape[0]
    if c1w < 8 or c1w % 8 or 256 % (c1w // 4) or c2w % 8:
        raise NotImplementedError("dgx edge MLP: conv1 width a multiple of 8 dividing 1024, conv2 width a "
                                  "multiple of 8 (PositionEmbedding: 64, 128)")
    if cv1.weight.shape[1] != 2 * x.shape[1]:
        raise RuntimeError(f"dgx edge MLP: conv1 expects {cv1.weight.shape[1]} edge channels, input has C={x.shape[1]}")
    return _EdgeMLP2.apply(x, k, bn1, bn2, act1.negative_slope, act2.negative_slope, training,
                           cv1.weight, bn1.weight, bn1.bias, cv2.weight, bn2.weight, bn2.bias)
