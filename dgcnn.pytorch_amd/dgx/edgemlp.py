"""PositionEmbedding's per-edge MLP: reference models/layers.py:45-52.

Reference:
    e  = get_graph_feature(x, k)                      (B, 2C, N, k)   layers.py:45
    h1 = conv1(e)   Conv2d(2C,64) + BN2d + LeakyReLU   per edge        layers.py:17-18, 48
    t  = conv2(h1)  Conv2d(64,128) + BN2d + LeakyReLU  per edge        layers.py:19-20, 49
    t  = t.max(dim=-1)[0]                             (B, 128, N)     layers.py:52

Engine: one autograd node. The edge tensor e is never built: conv1 is
decomposed into PQ = X [W1;W2]^T (y_e = P_j + Q_i, as in the EdgeConv chain)
and its BN statistics come from the EdgeConv gather kernel.
* bf16 mode (the benchmarked path): ONE fused forward kernel per step builds
  each 16-edge h1 tile from the gathered P_j / Q_i rows in registers / LDS,
  runs conv2 on the MFMA, and keeps the max over k (value + slot) and the BN2
  statistics (emlp_fwd_kernel: h1 and z2 never reach HBM); ONE fused backward
  kernel recomputes h1 and z2, applies the BN2 backward, chains dH1 = W2^T dZ2
  on the MFMA, applies LReLU'/BN1 and accumulates dW2 (emlp_bwd_kernel: no z2,
  dZ2 or dH1 in HBM), then the in-edge scatter forms dP / dQ.
* fp32 parity mode: the unfused kernels — h1 written per edge row (E = B*N*k
  rows), conv2 on the engine's fp32 MFMA GEMM, max over k, dense dZ2, the two
  conv2 GEMMs (dH1, dW2), LReLU/BN1 backward in place and the deterministic
  gather over the kNN graph and its reverse for dP / dQ.
"""
import torch

from . import _native as nat
from . import cpu
from . import bn as bn_
from . import gemm as G
from . import precision as prec
from .edgeconv import debug_capture, edge_select, split_weight
from .ops import knn_raw, reduction_order

# bf16 mode, C1 = 64 / C2 = 128 (PositionEmbedding): one backward kernel for
# conv2 + LReLU/BN1 (dgx_edge_mlp_fused_bwd_bf16: z2, dZ2, dH1 and dW2 in
# registers / LDS, h1 rebuilt from PQ), so the forward does not store h1.
# False keeps the unfused GEMM path (dZ2 / dH1 / dW2 GEMMs over a stored h1).
FUSED_BWD = True


def _fused_bwd_ok(bf16, C1, C2, k):
    return FUSED_BWD and bf16 and C1 == 64 and C2 == 128 and k <= 64


def _capture(idx, PQ, st1, st2, ysel, arg, bf16, fused):
    """Debug capture (tests): the stage's routing inputs under "emlp" — the kNN
    graph, conv1's decomposed PQ and BN1 affine (h1's LeakyReLU signs follow
    from them), conv2's selected pre-BN value / slot and BN2 affine. ``fused``:
    h1 was built as fma(a1, P_j, fma(a1, Q_i, b1)) and fed to the MFMA in bf16
    (emlp_fwd_kernel); otherwise as fma(a1, P_j + Q_i, b1) (mlp_h1_kernel)."""
    dbg = debug_capture()
    if dbg is not None:
        dbg["emlp"] = {"idx": idx.clone(), "PQ": PQ.clone(), "a1": st1.scale.clone(), "b1": st1.shift.clone(),
                       "ysel": ysel.clone(), "arg": arg.clone(), "a2": st2.scale.clone(), "b2": st2.shift.clone(),
                       "bf16": bf16, "fused": fused}


class _EdgeMLP2(torch.autograd.Function):
    @staticmethod
    @prec.no_autocast
    def forward(ctx, x, k, bn1, bn2, slope1, slope2, need_grad, knn_src, bf16, w1, g1, b1, w2, g2, b2):
        # the GEMM precision the caller's entry resolved (precision.effective: bf16 mode or autocast)
        with prec.mode("bf16" if bf16 else "fp32"):
            return _EdgeMLP2._forward(ctx, x, k, bn1, bn2, slope1, slope2, need_grad, knn_src, w1, g1, b1, w2, g2, b2)

    @staticmethod
    def _forward(ctx, x, k, bn1, bn2, slope1, slope2, need_grad, knn_src, w1, g1, b1, w2, g2, b2):
        x = x.float()
        dev = x.device
        B, C, N = x.shape
        M, E = B * N, B * N * k
        C1, C2 = w1.shape[0], w2.shape[0]
        L = nat.lib()
        stream = nat.stream_of(x)
        bf16 = prec.get() == "bf16"
        X = x.permute(0, 2, 1).reshape(M, C).contiguous()  # B = 1 reshapes to a column-major view
        kx = x if knn_src is None else knn_src.float()                            # neighbours found on kx
        idx = knn_raw(kx, k, order=reduction_order(kx), out_dtype=torch.int32)   # layers.py:45 -> dgcnn.py:21
        w1s = split_weight(w1, C, C1)
        if C <= G.SMALLK_MAX:  # raw coordinates (K = 3): exact fp32 in every mode
            PQ = G.mm_smallk(X, w1s)                                              # (M, 2C1)
        else:
            PQ = G.mm_xwt(X, w1s) if bf16 else prec.mm(X, w1s.t())
        W2 = w2.reshape(C2, C1)
        use1, _ = bn_.mode(bn1)
        use2, _ = bn_.mode(bn2)
        with torch.cuda.device(dev):
            # ---- conv1: BN1 statistics over all E edges, then h1 per edge row
            if use1:
                _, _, sumP1, part1, prow = edge_select(PQ, idx, B, N, k, C1, g1, stream)
                st1 = bn_.batch_stats(part1, prow, float(E), bn1, g1, b1, stream)
            else:
                st1 = bn_.running_stats(bn1, g1, b1, stream)
                # sum_k P_j only enters the train-mode BN1 backward (c1 = 0 here)
                sumP1 = torch.zeros((M, C1), dtype=torch.float32, device=dev) if need_grad else None
            fused = bf16 and C1 == 64 and C2 in (64, 128) and k <= 64
            if fused:
                # h1 -> conv2 (MFMA) -> max over k + BN2 statistics in one kernel: z2 never
                # reaches HBM; h1 (bf16) is written only when the backward needs it
                wprep = G.prep_weight(w2, C2, C1, False)
                dir2 = torch.where(g2 < 0, -1.0, 1.0).to(torch.float32).contiguous()
                W2d = (W2 * dir2.view(C2, 1)).to(torch.bfloat16).contiguous()
                # h1 (bf16) for the unfused backward's GEMMs; the fused backward rebuilds it
                keep_h1 = need_grad and not _fused_bwd_ok(bf16, C1, C2, k)
                H1 = torch.empty((E, C1), dtype=torch.bfloat16, device=dev) if keep_h1 else None
                rows2 = L.dgx_edge_mlp_fused_rows(B, N)
                part2 = torch.empty((rows2, 2, C2), dtype=torch.float32, device=dev)
                ysel = torch.empty((M, C2), dtype=torch.float32, device=dev)
                arg = torch.empty((M, C2), dtype=torch.uint8, device=dev)
                nat.check(L.dgx_edge_mlp_fused_fwd_bf16(
                    nat.f32(PQ), 2 * C1, nat.i32(idx), B, N, k, C1, C2, nat.f32(st1.scale), nat.f32(st1.shift),
                    float(slope1), nat.bf16(W2d), nat.f32(dir2), nat.f32(ysel), nat.u8(arg), nat.f32(part2), rows2,
                    nat.ptr(H1, nat.BF16), stream), "edge mlp fused forward")
                st2 = (bn_.batch_stats(part2, rows2, float(E), bn2, g2, b2, stream) if use2
                       else bn_.running_stats(bn2, g2, b2, stream))
                # LReLU(BN2) of the selected values, written (B, C2, N) contiguous as the
                # reference's max over k returns it (LDS-transposed apply)
                out = torch.empty((B, C2, N), dtype=torch.float32, device=dev)
                nat.check(L.dgx_pointconv_apply_f32(nat.f32(ysel), C2, B, N, C2, nat.f32(st2.scale),
                                                    nat.f32(st2.shift), float(slope2), nat.f32(out), stream),
                          "bn apply")
                _capture(idx, PQ, st1, st2, ysel, arg, bf16, fused=True)
                ctx.dims = (B, C, N, k, C1, C2)
                ctx.slopes = (float(slope1), float(slope2))
                ctx.st = (st1, st2)
                ctx.wprep = wprep
                ctx.bf16 = bf16
                if need_grad:
                    ctx.save_for_backward(X, idx, PQ, sumP1, H1, None, ysel, arg, w1, w2)
                return out
            h16 = bf16 and C1 % 64 == 0
            H1 = torch.empty((E, C1), dtype=torch.bfloat16 if h16 else torch.float32, device=dev)
            nat.check(L.dgx_edge_mlp_h1_f32(nat.f32(PQ), 2 * C1, nat.i32(idx), B, N, k, C1, nat.f32(st1.scale),
                                            nat.f32(st1.shift), float(slope1), nat.ptr(H1, nat.F32, nat.BF16),
                                            int(h16), stream), "edge h1")
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
                    nat.check(L.dgx_colstats_f32(nat.f32(Z2), C2, E, C2, nat.f32(part2), rows, stream), "colstats")
            z16 = Z2.dtype == torch.bfloat16
            if use2:
                st2 = bn_.batch_stats(part2, part2.shape[0], float(E), bn2, g2, b2, stream)
            else:
                st2 = bn_.running_stats(bn2, g2, b2, stream)
            # ---- max over k (layers.py:52) of LReLU(BN2(z2)): select, then apply
            ysel = torch.empty((M, C2), dtype=torch.float32, device=dev)
            arg = torch.empty((M, C2), dtype=torch.uint8, device=dev)
            nat.check(L.dgx_edge_mlp_max_f32(nat.ptr(Z2, nat.F32, nat.BF16), int(z16), B, N, k, C2, nat.f32(st2.scale),
                                             nat.f32(ysel), nat.u8(arg), stream), "edge max")
            out = torch.empty((B, C2, N), dtype=torch.float32, device=dev)
            nat.check(L.dgx_pointconv_apply_f32(nat.f32(ysel), C2, B, N, C2, nat.f32(st2.scale), nat.f32(st2.shift),
                                                float(slope2), nat.f32(out), stream), "bn apply")
        _capture(idx, PQ, st1, st2, ysel, arg, bf16, fused=False)
        ctx.dims = (B, C, N, k, C1, C2)
        ctx.slopes = (float(slope1), float(slope2))
        ctx.st = (st1, st2)
        ctx.wprep = wprep
        ctx.bf16 = bf16
        if need_grad:
            ctx.save_for_backward(X, idx, PQ, sumP1, H1, Z2, ysel, arg, w1, w2)
        return out

    @staticmethod
    @prec.no_autocast
    def backward(ctx, dout):
        with prec.mode("bf16" if ctx.bf16 else "fp32"):
            grads = _EdgeMLP2._backward(ctx, dout)
        return grads[:8] + (None,) + tuple(grads[8:])

    @staticmethod
    def _backward(ctx, dout):
        st1, st2 = ctx.st
        X, idx, PQ, sumP1, H1, Z2, ysel, arg, w1, w2 = ctx.saved_tensors
        B, C, N, k, C1, C2 = ctx.dims
        slope1, slope2 = ctx.slopes
        M, E = B * N, B * N * k
        dev = X.device
        L = nat.lib()
        stream = nat.stream_of(X)
        fused = Z2 is None  # fused forward: z2 was never stored
        fused_bwd = fused and H1 is None  # ... and h1 neither: the fused backward kernel
        z16 = fused or Z2.dtype == torch.bfloat16
        dout = dout.float()
        dY_pm = dout.permute(0, 2, 1)  # (B, N, C2): point-major if the gradient came that way
        with torch.cuda.device(dev):
            # ---- BN2 + LReLU backward at the selected edges, then dense over all edges
            dz = torch.empty((M, C2), dtype=torch.float32, device=dev)
            if dY_pm.is_contiguous():
                nblk = max(1, min(1024, (M + 63) // 64))
                part = torch.empty((nblk, 2, C2), dtype=torch.float32, device=dev)
                nat.check(L.dgx_edge_bwd_dz_f32(nat.f32(dY_pm), C2, nat.f32(ysel), M, C2, nat.f32(st2.scale),
                                                nat.f32(st2.shift), nat.f32(st2.mean), nat.f32(st2.invstd), slope2,
                                                nat.f32(dz), nat.f32(part), nblk, stream), "edge bwd dz")
            else:  # (B, C2, N) gradient (a contiguous downstream): read channel-major, no transpose copy
                dcm = dout.contiguous()
                nblk = L.dgx_edge_bwd_dz_cm_rows(B, N)
                part = torch.empty((nblk, 2, C2), dtype=torch.float32, device=dev)
                nat.check(L.dgx_edge_bwd_dz_cm_f32(nat.f32(dcm), nat.f32(ysel), B, N, C2, nat.f32(st2.scale),
                                                   nat.f32(st2.shift), nat.f32(st2.mean), nat.f32(st2.invstd),
                                                   slope2, nat.f32(dz), nat.f32(part), nblk, stream), "edge bwd dz")
            dg2, db2, c0, c1 = bn_.backward_consts(part, nblk, float(E), st2, stream)
            if fused_bwd:
                # conv2 + LReLU/BN1 backward in one pass: gE, BN1 partials, dW2 slabs
                rows = L.dgx_edge_mlp_fused_bwd_rows(B, N)
                part1 = torch.empty((rows, 2, C1), dtype=torch.float32, device=dev)
                slab = torch.empty((rows, C2, C1), dtype=torch.float32, device=dev)
                gE = torch.empty((E, C1), dtype=torch.bfloat16, device=dev)
                consts = torch.cat([c0, c1, st2.scale]).contiguous()
                nat.check(L.dgx_edge_mlp_fused_bwd_bf16(
                    nat.f32(PQ), 2 * C1, nat.i32(idx), B, N, k, C1, C2, nat.f32(st1.scale), nat.f32(st1.shift),
                    nat.f32(st1.mean), nat.f32(st1.invstd), slope1, nat.bf16(ctx.wprep[0]), nat.f32(dz), nat.u8(arg),
                    nat.f32(consts), nat.bf16(gE), nat.f32(part1), nat.f32(slab), rows, stream), "edge mlp fused bwd")
                gw2 = torch.empty((C2, C1), dtype=torch.float32, device=dev)
                nat.check(L.dgx_slab_reduce_f32(nat.f32(slab), rows, C2, C1, C2, nat.f32(gw2), C1, stream),
                          "dW2 slab reduce")
                g16 = 1
            elif fused:
                # z2 recomputed from h1 on the MFMA, BN2 backward in the GEMM's epilogue:
                # dZ2 = c1 z2 + c0 + [slot] a2 dz, stored bf16 (z2 never reaches HBM)
                dZ2 = torch.empty((E, C2), dtype=torch.bfloat16, device=dev)
                consts = torch.cat([c0, c1, st2.scale]).contiguous()
                nat.check(L.dgx_gemm_dz2_bf16(nat.bf16(H1), nat.bf16(ctx.wprep[0]), E, C2, C1, nat.f32(dz),
                                              nat.u8(arg), nat.f32(consts), k, nat.bf16(dZ2), stream), "edge dz2 gemm")
            else:
                dZ2 = torch.empty((E, C2), dtype=Z2.dtype, device=dev)
                nat.check(L.dgx_edge_mlp_dz_f32(nat.f32(dz), nat.u8(arg), nat.ptr(Z2, nat.F32, nat.BF16), int(z16), B, N,
                                                k, C2, nat.f32(st2.scale), nat.f32(c0), nat.f32(c1),
                                                nat.ptr(dZ2, nat.F32, nat.BF16), stream), "edge dz2")
            # ---- conv2 GEMMs: dH1 = dZ2 W2, dW2 = dZ2^T H1; then LReLU + BN1 backward
            if fused_bwd:
                pass
            elif ctx.wprep is not None and z16 and C1 == 64:
                gw2 = torch.empty((C2, C1), dtype=torch.float32, device=dev)
                # dH1 never leaves the GEMM tile: its epilogue forms g = dH1 LReLU'(z1) (bf16)
                # and the BN1-backward column partials
                G.lds_atb(dZ2, H1, gw2)
                rows = L.dgx_gemm_h1bwd_rows(E)
                part1 = torch.empty((rows, 2, C1), dtype=torch.float32, device=dev)
                gE = torch.empty((E, C1), dtype=torch.bfloat16, device=dev)
                nat.check(L.dgx_gemm_h1bwd_bf16(
                    nat.bf16(dZ2), nat.bf16(ctx.wprep[1]), E, C1, C2, nat.f32(PQ), 2 * C1, nat.i32(idx), N, k,
                    nat.f32(st1.scale), nat.f32(st1.shift), nat.f32(st1.mean), nat.f32(st1.invstd), slope1,
                    nat.bf16(gE), nat.f32(part1), rows, stream), "edge h1 bwd gemm")
                g16 = 1
            else:
                gw2 = torch.empty((C2, C1), dtype=torch.float32, device=dev)
                if ctx.wprep is not None and z16:
                    gE = G.lds_xwt(dZ2, ctx.wprep[1])
                    G.lds_atb(dZ2, H1, gw2)
                else:
                    W2 = w2.reshape(C2, C1)
                    gE = prec.mm(dZ2.float(), W2)
                    gw2 = prec.mm(dZ2.float().t(), H1.float())
                rows = L.dgx_edge_mlp_h1_bwd_rows(B, N, k, C1)
                part1 = torch.empty((rows, 2, C1), dtype=torch.float32, device=dev)
                nat.check(L.dgx_edge_mlp_h1_bwd_f32(nat.f32(gE), nat.f32(PQ), 2 * C1, nat.i32(idx), B, N, k, C1,
                                                    nat.f32(st1.scale), nat.f32(st1.shift), nat.f32(st1.mean),
                                                    nat.f32(st1.invstd), slope1, nat.f32(part1), rows, stream),
                          "edge h1 bwd")
                g16 = 0
            dg1, db1, e0, e1 = bn_.backward_consts(part1, rows, float(E), st1, stream)
            # ---- dP / dQ over the graph
            rowptr = torch.empty(M + 1, dtype=torch.int32, device=dev)
            edges = torch.empty(E, dtype=torch.int32, device=dev)
            nat.check(L.dgx_graph_reverse(nat.i32(idx), B, N, k, nat.i32(rowptr), nat.i32(edges), stream),
                      "reverse graph")
            dPQ = torch.empty((M, 2 * C1), dtype=torch.float32, device=dev)
            nat.check(L.dgx_edge_mlp_scatter_f32(nat.ptr(gE, nat.F32, nat.BF16), g16, nat.f32(PQ), 2 * C1,
                                                 nat.f32(sumP1), nat.i32(rowptr), nat.i32(edges), B, N, k, C1,
                                                 nat.f32(st1.scale), nat.f32(e0), nat.f32(e1), nat.f32(dPQ), stream),
                      "edge h1 scatter")
        # ---- conv1 (K = C, tiny): dW1 = [dP^T X | dQ^T X], dX = dP W1a + dQ W1b
        dx = None
        if ctx.bf16:  # the engine's GEMMs (split-K over the M rows, un-stacked in the slab sum)
            gw1 = torch.empty((C1, 2 * C), dtype=torch.float32, device=dev)
            G.mm_atb(dPQ, X, gw1, split_rows=C1)
            gw1 = gw1.view(w1.shape)
            if ctx.needs_input_grad[0]:
                dx = G.mm_xw(dPQ, split_weight(w1, C, C1)).view(B, N, C).permute(0, 2, 1)
        else:
            dwcat = prec.mm(dPQ.t(), X)  # (2C1, C)
            gw1 = torch.cat([dwcat[:C1], dwcat[C1:]], dim=1).reshape(w1.shape)
            if ctx.needs_input_grad[0]:
                dx = prec.mm(dPQ, split_weight(w1, C, C1)).view(B, N, C).permute(0, 2, 1)
        return (dx, None, None, None, None, None, None, None, gw1, dg1, db1, gw2.view(w2.shape), dg2, db2)


def edge_mlp2(x, k, conv1, conv2, training=None, knn_src=None):
    """max_k conv2(conv1(get_graph_feature(x, k))) for conv1/conv2 =
    nn.Sequential(Conv2d(1x1, bias=False), BatchNorm2d, LeakyReLU) as
    PositionEmbedding builds them (reference models/layers.py:17-20, 45-52).
    Returns (B, C2, N) contiguous, as the reference's max over k.
    ``training`` is accepted for call compatibility only (dgx.bn: each BN
    module's own flags decide batch vs running statistics). ``knn_src``:
    optional (B, C', N) tensor the neighbours are searched on instead of x
    (upstream's dim9 semseg graph: kNN on the normalised xyz channels).
    A host tensor takes the CPU path (dgx.cpu)."""
    if cpu.is_cpu(x):
        return cpu.edge_mlp2(x, k, conv1, conv2, training, knn_src)
    nat.require_device(x)
    if torch.compiler.is_compiling():   # traced as one dgx::edge_mlp2 op (dgx.library)
        from . import library
        return library.edge_mlp2_call(x, k, conv1, conv2, knn_src)
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
    params = (cv1.weight, bn1.weight, bn1.bias, cv2.weight, bn2.weight, bn2.bias)
    need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
    if knn_src is not None:
        nat.require_device(knn_src)
        knn_src = knn_src.detach()
        if knn_src.shape[0] != x.shape[0] or knn_src.shape[2] != x.shape[2]:
            raise RuntimeError("dgx edge MLP: knn_src must be (B, C', N) with the input's B and N")
    bf16 = prec.effective() == "bf16"
    return _EdgeMLP2.apply(x, k, bn1, bn2, act1.negative_slope, act2.negative_slope, need_grad, knn_src, bf16,
                           *params)
