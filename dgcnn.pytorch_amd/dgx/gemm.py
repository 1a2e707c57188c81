"""Host side of the engine's bf16 MFMA GEMMs (csrc/gemm.hip, C ABI dgx_gemm_bf16).

Every GEMM of the chain is ``C[i][j] = sum_k opA(i,k) opB(j,k)`` with each
operand either k-contiguous ("kc": row i at A[i*ld:]) or i-contiguous ("ic":
column i of a row-major (K, ld) buffer). Operands are fp32 or bf16 views of
existing buffers (column slices of the concat buffer included): nothing is
copied or converted on the host side.
"""
import threading

import torch

from . import _native as nat

EPI_STORE, EPI_ACCUM, EPI_STATS, EPI_SLAB, EPI_STATS16 = 0, 1, 2, 3, 4

# Optional per-thread instrumentation (tools): when a list, every GEMM launch
# of this thread appends (start_event, end_event, flops, tag) recorded on the
# launch stream. Per thread, so nn.DataParallel replicas (one Python thread per
# device) never record into each other's lists.
_tls = threading.local()


def set_timing(lst):
    _tls.timing = lst


class _Timed:
    def __init__(self, flops):
        self.flops = flops
        self.timing = getattr(_tls, "timing", None)

    def __enter__(self):
        if self.timing is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if self.timing is not None:
            self.e1.record()
            self.timing.append((self.e0, self.e1, self.flops, getattr(_tls, "tag", None)))
        return False


class tag:
    """Label the GEMM launches issued inside (this thread only)."""
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.prev = getattr(_tls, "tag", None)
        _tls.tag = self.name
        return self

    def __exit__(self, *exc):
        _tls.tag = self.prev
        return False


def _operand(t, ic):
    """(pointer, is_bf16, ld) of a 2-D view whose inner dim is unit-stride."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise RuntimeError(f"dgx gemm: operand must be a 2-D row-major view, got strides {t.stride()}")
    if t.dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError(f"dgx gemm: operand dtype {t.dtype} (fp32/bf16 only)")
    ld = t.stride(0) if t.shape[0] > 1 else max(1, t.shape[1])
    return nat.ptr(t), int(t.dtype == torch.bfloat16), int(ic), ld


def gemm(a, a_ic, b, b_ic, M, N, K, epi, out, partials=None, splits=1):
    """Raw launch. ``a``: (M,K) view if not a_ic else (K,M); same for ``b`` with N."""
    ap, abf, aic, lda = _operand(a, a_ic)
    bp, bbf, bic, ldb = _operand(b, b_ic)
    if epi == EPI_SLAB:
        ldc = N
    else:
        if out.dim() != 2 or out.stride(1) != 1 or out.dtype != torch.float32:
            raise RuntimeError("dgx gemm: output must be a row-major fp32 2-D view")
        ldc = out.stride(0)
    with torch.cuda.device(out.device), _Timed(2.0 * M * N * K):
        nat.check(nat.lib().dgx_gemm_bf16(ap, abf, aic, lda, bp, bbf, bic, ldb, M, N, K, epi, splits,
                                          nat.ptr(out), ldc, nat.ptr(partials), nat.stream_of(out)), "gemm bf16")
    return out


def mm_xwt(x, w, out=None, stats=False):
    """out (M,N) = x (M,K) @ w (N,K)^T; with ``stats`` also returns the column
    partials (rows, 2, N) of the train-mode BatchNorm statistics."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    part = None
    if stats:
        part = torch.empty((nat.lib().dgx_gemm_stats_rows(M), 2, N), dtype=torch.float32, device=x.device)
    gemm(x, False, w, False, M, N, K, EPI_STATS if stats else EPI_STORE, out, part)
    return (out, part) if stats else out


def _op32(t, contiguous_dim):
    """(tensor, ic, ld) reading a 2-D fp32 view in place: ``contiguous_dim`` 1
    means "k" is dim 1 (opA(i,k) = t[i,k]), 0 means "k" is dim 0 (opB(j,k) =
    t[k,j]); falls back to a contiguous copy for a view with no unit stride."""
    if t.dtype != torch.float32:
        t = t.float()
    kd, od = contiguous_dim, 1 - contiguous_dim
    if t.stride(kd) == 1 or t.shape[kd] == 1:            # k contiguous: KC, ld = stride of the other dim
        return t, 0, max(t.stride(od), t.shape[kd], 1) if t.shape[od] > 1 else max(t.shape[kd], 1)
    if t.stride(od) == 1 or t.shape[od] == 1:            # rows contiguous: IC, ld = stride along k
        return t, 1, max(t.stride(kd), t.shape[od], 1) if t.shape[kd] > 1 else max(t.shape[od], 1)
    t = t.contiguous() if kd == 1 else t.t().contiguous().t()
    return _op32(t, contiguous_dim)


def mm32(a, b, out=None, accumulate=False, addend=None):
    """out (M,N) = a (M,K) @ b (K,N) on the engine's fp32 MFMA GEMM
    (dgx_gemm_f32, exact fp32 products): the parity mode's GEMMs. Transposed
    views are read in place; a long reduction (K >= 2048 over few outputs,
    the weight gradients over B*N rows) is split over workgroups into slabs
    summed in a fixed order (deterministic). ``accumulate``: out += a @ b;
    ``addend``: out = addend + a @ b."""
    M, K = a.shape
    N = b.shape[1]
    if b.shape[0] != K:
        raise RuntimeError(f"dgx mm32: inner dims {K} and {b.shape[0]} differ")
    if accumulate and out is None:
        raise RuntimeError("dgx mm32: accumulate=True needs an output to accumulate into")
    ta, aic, lda = _op32(a, 1)
    tb, bic, ldb = _op32(b, 0)
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    if out.dtype != torch.float32 or out.dim() != 2 or (out.stride(1) != 1 and N > 1):
        raise RuntimeError("dgx mm32: output must be a row-major fp32 2-D view")
    L = nat.lib()
    S = L.dgx_gemm_f32_splits(M, N, K) if (K >= 2048 and not accumulate and addend is None) else 1
    st = nat.stream_of(out)
    with torch.cuda.device(out.device), _Timed(2.0 * M * N * K):
        if S > 1:
            kchunk = -(-K // S)
            kchunk = -(-kchunk // 16) * 16
            used = -(-K // kchunk)
            slab = torch.empty((used, M, N), dtype=torch.float32, device=out.device)
            nat.check(L.dgx_gemm_f32(nat.ptr(ta), aic, lda, nat.ptr(tb), bic, ldb, M, N, K, EPI_SLAB, S,
                                     nat.ptr(slab), N, None, 0, st), "gemm f32 (split-K)")
            nat.check(L.dgx_slab_reduce_f32(nat.ptr(slab), used, M, N, M, nat.ptr(out), out.stride(0), st),
                      "slab reduce")
        else:
            epi = EPI_ACCUM if (accumulate or addend is not None) else EPI_STORE
            nat.check(L.dgx_gemm_f32(nat.ptr(ta), aic, lda, nat.ptr(tb), bic, ldb, M, N, K, epi, 1, nat.ptr(out),
                                     out.stride(0) if M > 1 else max(N, 1), nat.ptr(addend),
                                     addend.stride(0) if addend is not None else 0, st), "gemm f32")
    return out


def mm16(a, b, out=None, accumulate=False):
    """out (M,N) (+)= a (M,K) @ b (K,N) on the bf16 MFMA GEMM (dgx_gemm_bf16:
    fp32 or bf16 operands rounded to bf16 while staged, fp32 accumulation);
    transposed views read in place; long reductions split-K (deterministic)."""
    if accumulate and out is None:
        raise RuntimeError("dgx mm16: accumulate=True needs an output to accumulate into")
    M, K = a.shape
    N = b.shape[1]
    if a.stride(1) != 1 and a.stride(0) != 1:
        a = a.contiguous()
    if b.stride(1) != 1 and b.stride(0) != 1:
        b = b.contiguous()
    a_ic = a.stride(1) != 1           # (M,K) with unit stride along M: pass a^T (K,M) row-major
    b_ic = b.stride(1) == 1           # (K,N) row-major: opB(j,k) = b[k,j] is j-contiguous
    A = a.t() if a_ic else a
    Bv = b if b_ic else b.t()
    if K >= 2048 and not accumulate and out is None and a_ic and b_ic:
        # the weight-gradient form (reduction over the B*N rows): split-K slabs
        o = torch.empty((M, N), dtype=torch.float32, device=a.device)
        return mm_atb(A, Bv, o)
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    gemm(A, a_ic, Bv, b_ic, M, N, K, EPI_ACCUM if accumulate else EPI_STORE, out)
    return out


SMALLK_MAX = 16


def mm_smallk(x, w):
    """Exact fp32 (M,N) = x (M,K) @ w (N,K)^T for K <= 16 (dgx_gemm_smallk_f32):
    the layer-1 GEMM on raw coordinates, exact in every precision mode."""
    M, K = x.shape
    N = w.shape[0]
    if x.stride(1) != 1:
        x = x.contiguous()
    w = w.contiguous()
    out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    with torch.cuda.device(x.device), _Timed(2.0 * M * N * K):
        nat.check(nat.lib().dgx_gemm_smallk_f32(nat.f32(x), x.stride(0) if M > 1 else K, nat.f32(w), M, N, K,
                                                nat.f32(out), N, nat.stream_of(x)), "gemm small-k")
    return out


def mm_smallk_split(x, wref, co):
    """mm_smallk(x, [W1; W2]) for a conv weight wref (Co, 2K[,1,1]) = [W1 | W2]
    in the reference layout (dgx_gemm_smallk_split_f32): the EdgeConv PQ of the
    3-channel block, no reshuffled weight copy."""
    M, K = x.shape
    if x.stride(1) != 1:
        x = x.contiguous()
    w = wref.reshape(co, 2 * K)
    if not w.is_contiguous():
        w = w.contiguous()
    out = torch.empty((M, 2 * co), dtype=torch.float32, device=x.device)
    with torch.cuda.device(x.device), _Timed(2.0 * M * 2 * co * K):
        nat.check(nat.lib().dgx_gemm_smallk_split_f32(nat.f32(x), x.stride(0) if M > 1 else K, nat.f32(w), M, co, K,
                                                      nat.f32(out), 2 * co, nat.stream_of(x)), "gemm small-k")
    return out


def mm_xw(x, w, out=None, accumulate=False):
    """out (M,N) (+)= x (M,K) @ w (K,N)."""
    M, K = x.shape
    N = w.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    gemm(x, False, w, True, M, N, K, EPI_ACCUM if accumulate else EPI_STORE, out)
    return out


def mm_atb(a, b, out, split_rows=None):
    """out = a^T @ b for a (R, M), b (R, N) (reduction over the R rows, split-K
    over workgroups, deterministic slab sum). ``split_rows`` = Co un-stacks a
    [W1;W2] result into out = [W1 | W2] (out is (M - Co, 2N))."""
    R, M = a.shape
    N = b.shape[1]
    if out.dtype != torch.float32 or out.stride(1) != 1:
        raise RuntimeError("dgx gemm: output must be a row-major fp32 view")
    L = nat.lib()
    S = L.dgx_gemm_splits(M, N, R)
    slab = torch.empty((S, M, N), dtype=torch.float32, device=a.device)
    gemm(a, True, b, True, M, N, R, EPI_SLAB, slab, splits=S)
    # the launch may use fewer splits than asked when R is short; count them the same way
    chunk = -(-R // S)
    chunk = -(-chunk // 32) * 32
    used = -(-R // chunk)
    split = M if split_rows is None else split_rows
    with torch.cuda.device(out.device):
        nat.check(L.dgx_slab_reduce_f32(nat.ptr(slab), used, M, N, split, nat.ptr(out), out.stride(0),
                                        nat.stream_of(out)), "slab reduce")
    return out


# ---- bf16-operand path (LDS-DMA staging, dgx_gemm_lds_bf16) ------------------

def _bf16_2d(t):
    if t.dtype != torch.bfloat16 or t.dim() != 2 or t.stride(1) != 1:
        raise RuntimeError("dgx gemm (bf16 path): operands must be row-major bf16 2-D views")
    return t.stride(0) if t.shape[0] > 1 else max(8, t.shape[1])


def lds_xwt(x16, w16, out=None, stats=False, accumulate=False, addend=None, out_bf16=False):
    """out (M,N) = x16 (M,K) @ w16 (N,K)^T (bf16 operands, K % 64 == 0).
    A split weight w16 (N, 2K) = [W_hi | W_lo] (prep_weights(..., split=True))
    gives x16 (W_hi + W_lo)^T: the weight with 16 significant bits.
    ``stats``: also returns the BatchNorm column partials (rows, 2, N);
    with ``out_bf16`` the product is stored bf16 (stats from the fp32 sums).
    ``accumulate``: out += ...; with ``addend``: out = addend + ... ."""
    M, K = x16.shape
    N = w16.shape[0]
    Kw = w16.shape[1]
    if Kw not in (K, 2 * K):
        raise RuntimeError(f"dgx gemm: weight k extent {Kw} does not match the operand's {K}")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16 if out_bf16 else torch.float32, device=x16.device)
    if out.dtype != (torch.bfloat16 if out_bf16 else torch.float32) or out.stride(1) != 1:
        raise RuntimeError("dgx gemm: output view dtype/layout does not match the epilogue")
    if addend is not None and (addend.dtype != torch.float32 or addend.stride(1) != 1):
        raise RuntimeError("dgx gemm: addend must be a row-major fp32 view")
    part = None
    if stats:
        part = torch.empty((nat.lib().dgx_gemm_stats_rows(M), 2, N), dtype=torch.float32, device=x16.device)
    if out_bf16 and not stats:
        raise RuntimeError("dgx gemm: a bf16 product is only stored together with its statistics")
    epi = (EPI_STATS16 if out_bf16 else EPI_STATS) if stats else (
        EPI_ACCUM if (accumulate or addend is not None) else EPI_STORE)
    with torch.cuda.device(out.device), _Timed(2.0 * M * N * Kw):
        nat.check(nat.lib().dgx_gemm_lds_bf16(
            nat.ptr(x16), _bf16_2d(x16), nat.ptr(w16), _bf16_2d(w16), 0, M, N, Kw, K, epi, 1, nat.ptr(out),
            out.stride(0), nat.ptr(part), nat.ptr(addend), addend.stride(0) if addend is not None else 0,
            nat.stream_of(out)), "gemm lds nt")
    return (out, part) if stats else out


def lds_xwt_edge_dz(x16, w16, addend, ysel, arg, st, slope):
    """dY = addend + x16 @ w16^T with the previous EdgeConv block's LeakyReLU'
    applied in the epilogue (dgx_gemm_edge_dz_bf16): returns (packed dz|slot
    words (M, N) fp32, column partials (rows, 2, N), rows) — what
    dgx_edge_bwd_dz_packed_f32 would make from the stored dY."""
    M, K = x16.shape
    N = w16.shape[0]
    L = nat.lib()
    rows = L.dgx_gemm_edge_dz_rows(M, N)
    dz = torch.empty((M, N), dtype=torch.float32, device=x16.device)
    part = torch.empty((rows, 2, N), dtype=torch.float32, device=x16.device)
    if addend.dtype != torch.float32 or addend.stride(1) != 1:
        raise RuntimeError("dgx gemm: addend must be a row-major fp32 view")
    with torch.cuda.device(x16.device), _Timed(2.0 * M * N * K):
        nat.check(L.dgx_gemm_edge_dz_bf16(
            nat.ptr(x16), _bf16_2d(x16), nat.ptr(w16), _bf16_2d(w16), M, N, K, nat.f32(addend), addend.stride(0),
            nat.f32(ysel), nat.u8(arg), nat.f32(st.scale), nat.f32(st.shift), nat.f32(st.mean), nat.f32(st.invstd),
            float(slope), nat.f32(dz), nat.f32(part), rows, nat.stream_of(x16)), "gemm edge dz")
    return dz, part, rows


# cap (MiB) on the split-K slab of the small bf16 weight-gradient GEMMs (output
# < 1 MiB: the EdgeConv blocks' dW). Default 8: block 4's dW takes 32 splits
# instead of 128 (33.5 -> 8.4 MB of slab); measured at cfg2 1.3442 -> 1.3384
# ms/step (2 / 4 MB: 1.401 / 1.359, too few workgroups). DGX_SLAB_CAP_MB=0
# restores dgx_gemm_splits's own rule.
SLAB_CAP_MB = int(__import__("os").environ.get("DGX_SLAB_CAP_MB", "8"))


def lds_atb(a16, b16, out, split_rows=None):
    """out = a16^T @ b16 for a16 (R, M), b16 (R, N) bf16 (reduction over R rows,
    split-K slabs summed deterministically); ``split_rows`` as in mm_atb."""
    R, M = a16.shape
    N = b16.shape[1]
    if out.dtype != torch.float32 or out.stride(1) != 1:
        raise RuntimeError("dgx gemm: output must be a row-major fp32 view")
    L = nat.lib()
    S = L.dgx_gemm_splits(M, N, R)
    if SLAB_CAP_MB > 0 and M * N * 4 < (1 << 20):   # bound the slab traffic of small outputs
        S = max(1, min(S, (SLAB_CAP_MB << 20) // (M * N * 4)))
    chunk = -(-R // S)
    chunk = -(-chunk // 64) * 64
    used = -(-R // chunk)
    slab = torch.empty((used, M, N), dtype=torch.float32, device=a16.device)
    with torch.cuda.device(out.device):
        st = nat.stream_of(out)
        with _Timed(2.0 * M * N * R):
            nat.check(L.dgx_gemm_lds_bf16(nat.ptr(a16), _bf16_2d(a16), nat.ptr(b16), _bf16_2d(b16), 1, M, N, R, R,
                                          EPI_SLAB, S, nat.ptr(slab), N, None, None, 0, st), "gemm lds tn")
        split = M if split_rows is None else split_rows
        nat.check(L.dgx_slab_reduce_f32(nat.ptr(slab), used, M, N, split, nat.ptr(out), out.stride(0), st),
                  "slab reduce")
    return out


def prep_weight(w, rows, cols, stacked):
    """bf16 operand copies of a conv weight: (nt (R, cols), tn (cols, R)) with
    R = 2*rows for a stacked EdgeConv weight (rows = Co, cols = C)."""
    R = 2 * rows if stacked else rows
    nt = torch.empty((R, cols), dtype=torch.bfloat16, device=w.device)
    tn = torch.empty((cols, R), dtype=torch.bfloat16, device=w.device)
    with torch.cuda.device(w.device):
        nat.check(nat.lib().dgx_weight_prep_bf16(nat.f32(w), rows, cols, int(stacked), nat.ptr(nt), nat.ptr(tn),
                                                 nat.stream_of(w)), "weight prep")
    return nt, tn


def prep_layout(shapes):
    """Layout of prep_weights' shared bf16 buffer for (rows, cols, stacked,
    split) jobs: (total elements, [(nt offset, nt shape, tn offset, tn shape)])
    with every view 16-byte aligned."""
    total, out = 0, []
    for (r, c, st, sp) in shapes:
        R = 2 * r if st else r
        n_tn, n_nt = R * c, (2 if sp else 1) * R * c
        p_tn, p_nt = -(-n_tn // 8) * 8, -(-n_nt // 8) * 8
        out.append((total, (R, 2 * c if sp else c), total + p_nt, (c, R)))
        total += p_nt + p_tn
    return total, out


def prep_views(buf, shapes):
    """[(nt, tn)] views of a prep_weights buffer (prep_layout's layout)."""
    _, lay = prep_layout(shapes)
    return [(buf[o1:o1 + s1[0] * s1[1]].view(s1), buf[o2:o2 + s2[0] * s2[1]].view(s2)) for (o1, s1, o2, s2) in lay]


def prep_weights(jobs, buf=None):
    """prep_weight for several (w, rows, cols, stacked[, split]) jobs in one
    launch; the bf16 copies share one allocation (``buf``, prep_layout's size,
    or a fresh one). Returns [(nt, tn), ...]. ``split``: nt is (R, 2*cols) =
    [W_hi | W_lo] for lds_xwt's split-weight form; tn (the backward's operand)
    is W_hi^T either way."""
    import ctypes
    if not jobs:
        return []
    jobs = [tuple(j) + (False,) * (5 - len(j)) for j in jobs]
    dev = jobs[0][0].device
    shapes = [(r, c, st, sp) for (_, r, c, st, sp) in jobs]
    total, _ = prep_layout(shapes)
    if buf is None:
        buf = torch.empty(total, dtype=torch.bfloat16, device=dev)
    elif buf.numel() != total or buf.dtype != torch.bfloat16:
        raise RuntimeError("dgx weight prep: buffer does not match the jobs' layout")
    out = prep_views(buf, shapes)
    n = len(jobs)
    P = ctypes.c_void_p * n
    I = ctypes.c_int * n
    # host arrays kept in locals for the duration of the call
    if any(w.dtype != torch.float32 for (w, _, _, _, _) in jobs):
        raise RuntimeError("dgx weight prep: fp32 weights expected")
    W = P(*[w.data_ptr() for (w, _, _, _, _) in jobs])
    NT = P(*[o[0].data_ptr() for o in out])
    TN = P(*[o[1].data_ptr() for o in out])
    CO = I(*[r for (_, r, _, _, _) in jobs])
    CI = I(*[c for (_, _, c, _, _) in jobs])
    ST = I(*[int(st) | (2 * int(sp)) for (_, _, _, st, sp) in jobs])
    with torch.cuda.device(dev):
        nat.check(nat.lib().dgx_weight_prep_multi_bf16(
            n, ctypes.addressof(W), ctypes.addressof(CO), ctypes.addressof(CI), ctypes.addressof(ST),
            ctypes.addressof(NT), ctypes.addressof(TN), nat.stream_of(jobs[0][0])), "weight prep")
    return out


def lds_ok_nt(x, K):
    """Whether the DMA path takes this k-contiguous operand (else the register-staged kernel)."""
    return x.dtype == torch.bfloat16 and K % 64 == 0 and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0


def edge_dz_ok(dpq16, cin):
    """Whether dgx_gemm_edge_dz_bf16 takes this block's input-gradient GEMM
    (dX columns = cin, K = dPQ width): the kernel's own limits (cin a multiple
    of 8 and <= 128, K a multiple of its 64-deep K step, 16-byte rows);
    otherwise the caller keeps the dY + dz-pass path."""
    K = dpq16.shape[1]
    return (dpq16.dtype == torch.bfloat16 and cin % 8 == 0 and cin <= 128 and K % 64 == 0
            and dpq16.stride(0) % 8 == 0 and dpq16.data_ptr() % 16 == 0)
