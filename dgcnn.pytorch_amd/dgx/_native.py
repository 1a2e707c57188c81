"""ctypes binding of libdgx.so (the C ABI in include/dgx.h).

The product path has exactly one implementation — the HIP kernels in this
library. If the library is missing or a ROCm device is not available the ops
raise; there is no CPU or eager-PyTorch fallback.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DGX_LIB", os.path.join(_HERE, "libdgx.so"))

ORDER_STRIDED = 0
ORDER_VEC8X4 = 1
GF_CAT, GF_DISP, GF_KNN_ONLY, GF_DIFFCAT = 0, 1, 2, 3

_lock = threading.Lock()
_lib = None

_vp, _i64, _i32, _f32, _f64, _sz = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float,
                                    ctypes.c_double, ctypes.c_size_t)

# name -> argtypes (restype int unless listed in _RESTYPES)
_SIGS = {
    "dgx_version": [],
    "dgx_strerror": [_i32],
    "dgx_knn_workspace_bytes": [_i32, _i32, _i32],
    "dgx_knn_image_bytes": [_i32, _i32, _i32],
    "dgx_knn_kernel_name": [_i32, _i32, _i32],
    "dgx_bn_lrelu_apply_knn_image_f32": [_vp, _i32, _i32, _i32, _vp, _vp, _f32, _vp, _i32, _vp, _vp, _vp, _sz, _vp],
    "dgx_knn_prepare_f32": [_vp, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _sz, _vp],
    "dgx_knn_f32": [_vp, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _sz, _vp],
    "dgx_sqnorm_f32": [_vp, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _vp, _vp],
    "dgx_knn_generic_workspace_bytes": [_i32, _i32, _i32],
    "dgx_knn_generic_f32": [_vp, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _sz, _vp],
    "dgx_knn_select_f32": [_vp, _i64, _i64, _i64, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _sz, _vp],
    "dgx_graph_feature_f32": [_vp, _i64, _i64, _i64, _i32, _i32, _i32, _vp, _i32, _i32, _vp, _vp],
    "dgx_graph_feature_bwd_f32": [_vp, _i32, _i32, _i32, _vp, _i32, _i32, _vp, _vp],
    "dgx_graph_feature_bwd_csr_f32": [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp],
    "dgx_sgd_step_f32": [_i32, _vp, _vp, _vp, _vp, _f32, _f32, _f32, _f32, _i32, _i32, _i32, _vp],
    "dgx_edge_partials_rows": [_i32, _i32, _i32],
    "dgx_edge_fwd_gather_f32": [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "dgx_edge_fwd_eval_f32": [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _f32, _vp, _i32, _vp],
    "dgx_bn_finalize_f32": [_vp, _i32, _i32, _f64, _vp, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _vp, _vp, _vp, _vp],
    "dgx_bn_finalize_out_f32": [_vp, _i32, _i32, _f64, _vp, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _vp, _vp, _vp, _vp,
                                _vp, _vp, _vp],
    "dgx_bn_finalize_out_f64": [_vp, _i32, _i32, _f64, _vp, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _vp, _vp, _vp, _vp,
                                _vp, _vp, _vp],
    "dgx_bn_finalize_f64": [_vp, _i32, _i32, _f64, _vp, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _vp, _vp, _vp, _vp],
    "dgx_bn_bwd_finalize_f64": [_vp, _i32, _i32, _f64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "dgx_bn_eval_affine_f32": [_i32, _vp, _vp, _vp, _vp, _f64, _vp, _vp, _vp],
    "dgx_bn_lrelu_apply_f32": [_vp, _i32, _i32, _vp, _vp, _f32, _vp, _i32, _vp, _vp],
    "dgx_edge_bwd_dz_f32": [_vp, _i32, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _i32, _vp],
    "dgx_edge_bwd_dz_packed_f32": [_vp, _i32, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _i32, _vp],
    "dgx_edge_bwd_dz_cm_rows": [_i32, _i32],
    "dgx_edge_bwd_dz_cm_f32": [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _i32, _vp],
    "dgx_bn_bwd_finalize_f32": [_vp, _i32, _i32, _f64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "dgx_graph_reverse": [_vp, _i32, _i32, _i32, _vp, _vp, _vp],
    "dgx_graph_reverse_multi": [_i32, _vp, _i32, _i32, _i32, _vp, _vp, _vp],
    "dgx_edge_bwd_scatter_f32": [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp,
                                 _i32, _vp],
    "dgx_edge_bwd_scatter_fin_f32": [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _i32, _f64,
                                     _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp],
    "dgx_edge_bwd_scatter_packed_f32": [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp,
                                        _i32, _vp],
    "dgx_edge_bwd_scatter_push_f32": [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _i32,
                                      _f64, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp],
    "dgx_colstats_rows": [_i64],
    "dgx_colstats_f32": [_vp, _i32, _i64, _i32, _vp, _i32, _vp],
    "dgx_pointconv_apply_f32": [_vp, _i32, _i32, _i32, _i32, _vp, _vp, _f32, _vp, _vp],
    "dgx_pointconv_bwd_rows": [_i32, _i32],
    "dgx_pointconv_bwd_f32": [_vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp],
    "dgx_pointconv_input_grad": [_vp, _vp, _i32, _i64, _i32, _vp, _vp, _vp, _vp, _i32, _vp],
    "dgx_to_bf16": [_vp, _i64, _i64, _i32, _vp, _vp],
    "dgx_split_bf16": [_vp, _i64, _i64, _i32, _vp, _vp, _i64, _vp],
    "dgx_gemm_stats_rows": [_i32],
    "dgx_gemm_splits": [_i32, _i32, _i32],
    "dgx_gemm_edge_dz_rows": [_i32, _i32],
    "dgx_gemm_edge_dz_bf16": [_vp, _i64, _vp, _i64, _i32, _i32, _i32, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _f32,
                              _vp, _vp, _i32, _vp],
    "dgx_gemm_bf16": [_vp, _i32, _i32, _i64, _vp, _i32, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _vp,
                      _vp],
    "dgx_gemm_f32": [_vp, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp],
    "dgx_gemm_f32_splits": [_i32, _i32, _i32],
    "dgx_gemm_smallk_split_f32": [_vp, _i64, _vp, _i32, _i32, _i32, _vp, _i64, _vp],
    "dgx_gemm_smallk_f32": [_vp, _i64, _vp, _i32, _i32, _i32, _vp, _i64, _vp],
    "dgx_slab_reduce_f32": [_vp, _i32, _i32, _i32, _i32, _vp, _i64, _vp],
    "dgx_slab_reduce_multi_f32": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dgx_gemm_lds_bf16": [_vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _vp,
                          _i64, _vp],
    "dgx_weight_prep_bf16": [_vp, _i32, _i32, _i32, _vp, _vp, _vp],
    "dgx_weight_prep_multi_bf16": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dgx_weight_stack_multi_f32": [_i32, _vp, _vp, _vp, _vp, _vp],
    "dgx_pointconv_bf16_rows": [_i32, _i32],
    "dgx_pointconv_apply_bf16": [_vp, _i32, _i32, _i32, _vp, _vp, _f32, _vp, _vp],
    "dgx_pointconv_bwd_bf16": [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _i32, _vp],
    "dgx_pointconv_bwd_split_f32": [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp,
                                    _i32, _vp],
    "dgx_edge_mlp_h1_f32": [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _f32, _vp, _i32, _vp],
    "dgx_edge_mlp_max_f32": [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp],
    "dgx_edge_mlp_dz_f32": [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp],
    "dgx_edge_mlp_h1_bwd_rows": [_i32, _i32, _i32, _i32],
    "dgx_edge_mlp_h1_bwd_f32": [_vp, _vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _i32,
                                _vp],
    "dgx_edge_mlp_scatter_f32": [_vp, _i32, _vp, _i32, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp,
                                 _vp],
    "dgx_gemm_h1bwd_rows": [_i32],
    "dgx_gemm_h1bwd_bf16": [_vp, _vp, _i32, _i32, _i32, _vp, _i32, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp,
                            _vp, _i32, _vp],
    "dgx_hog_1x1_f32": [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp],
    "dgx_hog_1x1_sem_f32": [_vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp],
    "dgx_attn_fwd": [_i32] + [_vp, _i64, _i64, _i64, _i64] * 3 + [_vp, _i64, _i64, _i64, _vp, _i32, _i32, _i32,
                                                                   _i32, _i32, _f32, _f32, ctypes.c_uint64, _vp,
                                                                   _vp],
    "dgx_attn_bwd": [_i32] + [_vp, _i64, _i64, _i64, _i64] * 3 + [_vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp,
                                                                   _i32, _i32, _i32, _i32, _i32, _f32, _f32,
                                                                   ctypes.c_uint64, _vp]
                    + [_vp, _i64, _i64, _i64] * 3 + [_vp],
    "dgx_attn_dropout_mask": [_i64, _i32, _f32, ctypes.c_uint64, _vp, _vp],
    "dgx_edge_mlp_fused_rows": [_i32, _i32],
    "dgx_edge_mlp_fused_bwd_rows": [_i32, _i32],
    "dgx_edge_mlp_fused_bwd_bf16": [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "dgx_gemm_dz2_bf16": [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp],
    "dgx_edge_mlp_fused_fwd_bf16": [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _f32, _vp, _vp, _vp, _vp,
                                    _vp, _i32, _vp, _vp],
}
_RESTYPES = {
    "dgx_version": ctypes.c_char_p,
    "dgx_strerror": ctypes.c_char_p,
    "dgx_knn_kernel_name": ctypes.c_char_p,
    "dgx_knn_workspace_bytes": _sz,
    "dgx_knn_image_bytes": _sz,
    "dgx_knn_generic_workspace_bytes": _sz,
}


def exported_symbols():
    return sorted(_SIGS)


def lib():
    """Load libdgx.so once (thread-safe: nn.DataParallel calls ops from threads)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(
                        f"dgx: HIP library not built ({LIB_PATH}); run `make -C dgcnn.pytorch_amd/csrc` "
                        "or __graft_entry__.build()")
                handle = ctypes.CDLL(LIB_PATH)
                for name, argtypes in _SIGS.items():
                    fn = getattr(handle, name)
                    fn.argtypes = argtypes
                    fn.restype = _RESTYPES.get(name, ctypes.c_int)
                _lib = handle
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().dgx_strerror(rc).decode()
        raise RuntimeError(f"dgx: {what} failed ({rc}: {msg})")


def ptr(t, *dtypes):
    """Device pointer of ``t`` (None passes through). With ``dtypes`` the tensor
    must have one of them: every kernel argument's element type is fixed by the
    C ABI (include/dgx.h), and a tensor of another dtype (e.g. an fp16 product
    made under autocast) would be read with the wrong element size."""
    if t is None:
        return None
    if dtypes and t.dtype not in dtypes:
        raise RuntimeError(f"dgx: kernel operand has dtype {t.dtype}, expected {' or '.join(map(str, dtypes))}")
    return ctypes.c_void_p(t.data_ptr())


F32, BF16, I32, I64, U8, F64, F16 = (torch.float32, torch.bfloat16, torch.int32, torch.int64, torch.uint8,
                                    torch.float64, torch.float16)


def f32(t):
    return ptr(t, F32)


def bf16(t):
    return ptr(t, BF16)


def i32(t):
    return ptr(t, I32)


def u8(t):
    return ptr(t, U8)


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(*tensors):
    for t in tensors:
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
            raise RuntimeError("dgx ops run on ROCm device tensors only (MI355X); got "
                               f"{getattr(t, 'device', type(t))}")
