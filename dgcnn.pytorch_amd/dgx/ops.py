"""Device ops behind the reference's graph functions (models/dgcnn.py:6-44).

``knn`` and ``graph_feature`` keep the reference's argument meaning, return
shapes and dtypes; the work is done by libdgx.so on the tensor's own device
and current stream.
"""
import contextlib
import threading

import torch

from . import _native as nat
from . import cpu

_tls = threading.local()

def reduction_order(x):
    """Rounding order of the reference's ``sum(x**2, dim=1)`` (dgcnn.py:8) for a
    (B,C,N) tensor with these strides: torch reduces a channel-innermost layout
    with its vectorised inner reduction, an N-innermost one with the strided
    cascade (see oracle/knn_oracle.c, pinned by tests/golden)."""
    _, C, N = x.shape
    _, sC, sN = x.stride()
    if C > 1 and N > 1 and sC < sN:
        return nat.ORDER_VEC8X4
    return nat.ORDER_STRIDED


def _as_f32(x):
    # autocast may hand fp16/bf16 features; distances are always fp32
    return x if x.dtype == torch.float32 else x.float()


def knn_image_buffers(B, C, N, dev):
    """(xx, image) scratch of one kNN call (dgx_knn_prepare_f32's outputs); a
    producer kernel may fill them (dgx_bn_lrelu_apply_knn_image_f32) and hand
    them to knn_raw(prepared=...)."""
    L = nat.lib()
    img_bytes = L.dgx_knn_image_bytes(B, C, N)
    xx = torch.empty((B * N,), dtype=torch.float32, device=dev)
    img = torch.empty((max(img_bytes, 4) + 3) // 4, dtype=torch.float32, device=dev)
    return xx, img


# shapes of the fused selection kernel (csrc/knn.hip); the rest take the
# generic path (csrc/knn_generic.hip): same values, same canonical order
FAST_MAXC, FAST_MAXK, FAST_MAXN = 128, 64, 12288
GENERIC_MAXK = 8192


def fast_shape(C, k, N):
    return C <= FAST_MAXC and k <= FAST_MAXK and N <= FAST_MAXN


def _knn_generic(x, strides, shape, k, order, idx, vals, stream):
    """dgx_knn_generic_f32 on a (B,C,N) view; a view with neither inner
    stride 1 is read from a contiguous copy (the rounding order was taken from
    the caller's strides)."""
    B, C, N = shape
    sB, sC, sN = strides
    if k > GENERIC_MAXK:
        raise NotImplementedError(f"dgx knn: k = {k} > {GENERIC_MAXK} neighbours")
    if sN != 1 and sC != 1:
        x = torch.as_strided(x, shape, strides).contiguous()
        sB, sC, sN = x.stride()
    L = nat.lib()
    ws_bytes = L.dgx_knn_generic_workspace_bytes(B, C, N)
    ws = torch.empty(((ws_bytes + 3) // 4,), dtype=torch.float32, device=x.device)
    i64 = idx.dtype == torch.int64
    with torch.cuda.device(x.device):
        nat.check(L.dgx_knn_generic_f32(nat.f32(x), sB, sC, sN, B, C, N, k, order,
                                        nat.ptr(idx, torch.int64) if i64 else None,
                                        nat.i32(idx) if not i64 else None, nat.f32(vals), nat.f32(ws), ws_bytes,
                                        stream), "knn (generic)")


def knn_raw(x, k, order=None, out_dtype=torch.int64, strides=None, shape=None, return_values=False, prepared=None):
    """kNN on a (B,C,N) fp32 view. ``strides``/``shape`` let callers describe a
    strided slice of a larger buffer (the engine's point-major concat buffer).
    ``prepared``: (xx, image) already holding |x|^2 in ``order`` and the operand
    image of exactly this view (knn_image_buffers + a producer kernel): the
    prepare pass is skipped."""
    nat.require_device(x)
    B, C, N = shape if shape is not None else x.shape
    sB, sC, sN = strides if strides is not None else x.stride()
    if order is None:
        order = reduction_order(x)
    if not (1 <= k <= N):
        raise RuntimeError(f"knn: selected index k out of range (k={k}, N={N})")
    generic = not fast_shape(C, k, N)
    if generic and prepared is not None:
        raise RuntimeError("knn: prepared operands exist for the fused kernel's shapes only")
    cache = getattr(_tls, "cache", None)
    key = None
    if cache is not None and not return_values:
        key = (x.device, x.data_ptr(), (B, C, N), (sB, sC, sN), x._version, k, order)
        hit = cache.get(key)
        if hit is not None:
            hit = hit[0]
            return hit if hit.dtype == out_dtype else hit.to(out_dtype)
    L = nat.lib()
    idx = torch.empty((B, N, k), dtype=out_dtype, device=x.device)
    vals = torch.empty((B, N, k), dtype=torch.float32, device=x.device) if return_values else None
    stream = nat.stream_of(x)
    if generic:
        _knn_generic(x, (sB, sC, sN), (B, C, N), k, order, idx, vals, stream)
        if key is not None:
            cache[key] = (idx, x)
        return (idx, vals) if return_values else idx
    img_bytes = L.dgx_knn_image_bytes(B, C, N)
    if prepared is not None:
        xx, img = prepared
        if xx.numel() != B * N or img.numel() * 4 < img_bytes:
            raise RuntimeError("knn: prepared |x|^2 / image buffers do not match the cloud")
    else:
        xx, img = knn_image_buffers(B, C, N, x.device)
    with torch.cuda.device(x.device):
        if prepared is None:
            # |x|^2 and the MFMA operand image in one pass over x
            nat.check(L.dgx_knn_prepare_f32(nat.f32(x), sB, sC, sN, B, C, N, order, nat.f32(xx), nat.f32(img),
                                            img_bytes, stream), "knn prepare")
        timing = getattr(_tls, "timing", None)
        if timing is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        rc = L.dgx_knn_select_f32(nat.f32(x), sB, sC, sN, nat.f32(xx), B, C, N, k,
                                  nat.ptr(idx, torch.int64) if out_dtype == torch.int64 else None,
                                  nat.i32(idx) if out_dtype == torch.int32 else None, nat.f32(vals),
                                  nat.f32(img), img_bytes, stream)
        if timing is not None:
            ev1.record()
            timing.append((ev0, ev1, 2.0 * B * N * N * C, (B, C, N, k)))
    nat.check(rc, "knn")
    if key is not None:
        # the entry holds x too: its storage (whose address is part of the key)
        # cannot be freed and reused by another tensor while the scope lives
        cache[key] = (idx, x)
    return (idx, vals) if return_values else idx


@contextlib.contextmanager
def knn_cache():
    """Scope in which kNN calls on the same view of the same storage (pointer,
    shape, strides, version counter) with the same k and rounding order share
    one computation. ``Net.forward`` reaches the kNN of its input cloud three
    times (reference model_partseg.py:177 -> dgcnn.py:84, :179 -> :26 and
    :183 -> layers.py:45); the result is a deterministic function
    of those keys, so the shared result is the one each call would compute.
    Each entry keeps its input tensor alive for the whole scope, so a storage
    address cannot be reused by another tensor inside it. Thread-local (DataParallel
    replicas run in threads)."""
    prev = getattr(_tls, "cache", None)
    _tls.cache = {} if prev is None else prev
    try:
        yield
    finally:
        _tls.cache = prev


class _Elapsed:
    """An already-measured launch (C++ HIP events), shaped like the
    (start_event, end_event) pair: start.elapsed_time(end) -> ms."""

    def __init__(self, ms):
        self.ms = ms

    def elapsed_time(self, _end):
        return self.ms


def set_knn_timing(lst):
    """Optional per-thread instrumentation (tools, bench.py's roofline leg):
    when a list, every kNN selection launch of this thread appends
    (start_event, end_event, gram_flops, shape) recorded on the launch stream —
    the Python dispatch's launches as they run, the C++ schedule's
    (libdgx_torch.so) when the timing is switched off again (set_knn_timing(None))."""
    prev = getattr(_tls, "timing", None)
    from . import host
    if lst is not None:
        host.load()
        torch.ops.dgx_host.knn_timing(True)
    elif prev is not None:
        v = torch.ops.dgx_host.knn_timing(False)
        for j in range(0, len(v), 6):
            prev.append((_Elapsed(v[j]), None, v[j + 1], (int(v[j + 2]), int(v[j + 3]), int(v[j + 4]), int(v[j + 5]))))
    _tls.timing = lst


def knn(x, k):
    """Drop-in for reference ``knn(x, k)`` (models/dgcnn.py:6-12): int64 (B,N,k)
    local indices, nearest first; ties in canonical (index ascending) order."""
    if torch.compiler.is_compiling():   # traced as one dgx::knn op (dgx.library)
        from . import library  # noqa: F401
        return torch.ops.dgx.knn(x, k)
    if cpu.is_cpu(x):   # host tensors: the CPU path (dgx.cpu), same canonical result
        return cpu.knn(x, k)
    x = _as_f32(x.detach())
    return knn_raw(x, k)


class _GraphFeature(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx32, mode):
        x = x.float()
        B, C, N = x.shape
        k = idx32.shape[-1]
        if mode in (nat.GF_CAT, nat.GF_DIFFCAT):
            out = torch.empty((B, 2 * C, N, k), dtype=torch.float32, device=x.device)
        elif mode == nat.GF_DISP:
            out = torch.empty((B, C, N, k), dtype=torch.float32, device=x.device)
        else:
            out = torch.empty((B, N, k, C), dtype=torch.float32, device=x.device)
        sB, sC, sN = x.stride()
        with torch.cuda.device(x.device):
            rc = nat.lib().dgx_graph_feature_f32(nat.f32(x), sB, sC, sN, B, C, N, nat.i32(idx32), k, mode,
                                                 nat.f32(out), nat.stream_of(x))
        nat.check(rc, "graph_feature")
        ctx.save_for_backward(idx32)
        ctx.mode = mode
        ctx.shape = (B, C, N)
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx32,) = ctx.saved_tensors
        B, C, N = ctx.shape
        dout = dout.contiguous().float()
        dx = torch.zeros((B, C, N), dtype=torch.float32, device=dout.device)
        k = idx32.shape[-1]
        with torch.cuda.device(dout.device):
            if k <= 64 and B * N < (1 << 25):
                # deterministic: pull over the reverse kNN graph (no float atomics)
                from .edgeconv import _reverse_graphs
                (rowptr, edges), = _reverse_graphs([idx32.contiguous()], B, N, k, dout.device)
                rc = nat.lib().dgx_graph_feature_bwd_csr_f32(nat.f32(dout), B, C, N, k, ctx.mode, nat.i32(rowptr),
                                                             nat.i32(edges), nat.f32(dx), nat.stream_of(dout))
            else:
                rc = nat.lib().dgx_graph_feature_bwd_f32(nat.f32(dout), B, C, N, nat.i32(idx32), k,
                                                         ctx.mode, nat.f32(dx), nat.stream_of(dout))
        nat.check(rc, "graph_feature backward")
        return dx, None, None


def graph_feature(x, k=20, knn_only=False, disp_only=False, idx=None, mode="cat"):
    """Drop-in for reference ``get_graph_feature`` (models/dgcnn.py:15-44).

    Default: (B,2C,N,k) fp32 contiguous, channels [0,C) = x_j, [C,2C) = x_i
    (dgcnn.py:42). knn_only: (B,N,k,C) neighbour rows (dgcnn.py:37-38).
    disp_only: (B,C,N,k) x_j - x_i (dgcnn.py:39-40). ``mode="diff"`` (engine
    extension): channels [0,C) = x_j - x_i, the paper's / test.ipynb:131 form.
    Differentiable w.r.t. x."""
    if mode not in ("cat", "diff"):
        raise ValueError(f"get_graph_feature: mode must be 'cat' or 'diff', got {mode!r}")
    diff = mode == "diff"
    mode = nat.GF_KNN_ONLY if knn_only else (nat.GF_DISP if disp_only else (nat.GF_DIFFCAT if diff else nat.GF_CAT))
    if torch.compiler.is_compiling() and idx is None:   # traced as one dgx::graph_feature op
        from . import library  # noqa: F401
        return torch.ops.dgx.graph_feature(x, k, mode)[0]
    if cpu.is_cpu(x):
        return cpu.graph_feature(x, k, knn_only, disp_only, idx, mode="diff" if diff else "cat")
    nat.require_device(x)
    x = _as_f32(x)
    if idx is None:
        idx = knn_raw(x.detach(), k, out_dtype=torch.int32)
    else:
        # caller-given ids (an engine extension): every kernel of the forward and
        # the reverse-graph backward assumes 0 <= id < N, so check once (one host
        # sync, only on this path); the reference's indexing raises likewise
        B, _, N = x.shape
        if idx.dim() != 3 or idx.shape[0] != B or idx.shape[1] != N:
            raise RuntimeError(f"get_graph_feature: idx of shape {tuple(idx.shape)} does not match x "
                               f"{tuple(x.shape)} (expected (B, N, k))")
        if idx.numel():
            lo, hi = torch.aminmax(idx.detach())
            if int(lo) < 0 or int(hi) >= N:
                raise IndexError(f"get_graph_feature: neighbour ids must lie in [0, {N}), got [{int(lo)}, {int(hi)}]")
        if idx.dtype != torch.int32:
            idx = idx.to(torch.int32)
    return _GraphFeature.apply(x, idx.contiguous(), mode)
