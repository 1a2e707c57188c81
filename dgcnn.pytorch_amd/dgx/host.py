"""Eager dispatch of DGCNN's train step through the C++ op layer
(libdgx_torch.so, csrc/dgx_torch.cpp): ``torch.ops.dgx_host.dgcnn_train``
runs the 4 EdgeConv blocks + conv5 forward (reference models/dgcnn.py:84-103)
and, from a C++ autograd node, their backward — the same libdgx.so kernels
with the same arguments as dgx.edgeconv / dgx.pointconv, so the results are
bit-identical; the ~60 launches of a step are issued from C++ instead of one
Python dispatch (ctypes conversion, tensor bookkeeping) each.

It serves the configuration the reference's training scripts run
(main_partseg_dist.py:253, main_cls.py): precision "bf16", every BatchNorm a
plain nn.BatchNorm2d in training mode tracking running statistics with a
momentum, gradients wanted. Anything else (fp32 parity mode, eval mode,
SyncBatchNorm, momentum=None, torch.compile tracing, instrumentation hooks)
takes the Python dispatch of the same kernels. ``DGX_HOST_EXT=0`` turns this
layer off (A/B runs); with it on, a missing libdgx_torch.so is an error.
"""
import os
import threading

import torch

from . import edgeconv as E
from . import gemm as G
from . import ops
from . import precision as prec

ENABLED = os.environ.get("DGX_HOST_EXT", "1") == "1"
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DGX_TORCH_LIB", os.path.join(_HERE, "libdgx_torch.so"))
_lock = threading.Lock()
_loaded = False


def load():
    """Register torch.ops.dgx_host (once)."""
    global _loaded
    if not _loaded:
        with _lock:
            if not _loaded:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(f"dgx: C++ op library not built ({LIB_PATH}); run `make -C "
                                      "dgcnn.pytorch_amd/csrc` or __graft_entry__.build() (DGX_HOST_EXT=0 skips it)")
                from . import _native
                _native.lib()   # libdgx.so first: libdgx_torch.so links against it
                torch.ops.load_library(LIB_PATH)
                _loaded = True


def _plain_train_bn(bn):
    return (type(bn) is torch.nn.BatchNorm2d and bn.training and bn.track_running_stats and bn.affine
            and bn.running_mean is not None and bn.momentum is not None)


def applies(model, x):
    """Whether DGCNN ``model``'s forward on ``x`` takes the C++ op."""
    if not ENABLED or prec.get() != "bf16" or torch.compiler.is_compiling():
        return False
    if x.device.type != "cuda" or x.dtype != torch.float32 or x.dim() != 3 or not torch.is_grad_enabled():
        return False
    if not (E.SCATTER_PACKED and E.FOLD_BN_BWD and E.FUSE_KNN_IMAGE and E.FUSE_EDGE_DZ and G.SLAB_CAP_MB == 8):
        return False
    if (E.debug_capture() is not None or getattr(G._tls, "timing", None) is not None
            or getattr(ops._tls, "timing", None) is not None):
        return False
    if model.k > 64 or model.k > x.shape[2] or tuple(model.WIDTHS) != (64, 64, 128, 256) or x.shape[1] > 16:
        return False
    seqs = model.edge_blocks() + [model.conv5]
    for seq in seqs:
        conv, bn = seq[0], seq[1]
        if conv.bias is not None or not _plain_train_bn(bn) or conv.weight.dtype != torch.float32:
            return False
    return any(seq[0].weight.requires_grad for seq in seqs) or x.requires_grad


def dgcnn_train(model, x):
    """DGCNN.forward (train mode) through torch.ops.dgx_host.dgcnn_train."""
    load()
    params, bufs, hyper = [], [], []
    weights = model.edge_weights() + [model.conv5[0].weight]   # re-parameterised in edge_mode "diff"
    for w, seq in zip(weights, model.edge_blocks() + [model.conv5]):
        conv, bn, act = seq[0], seq[1], seq[2]
        params += [w, bn.weight, bn.bias]
        bufs += [bn.running_mean, bn.running_var, bn.num_batches_tracked]
        hyper += [float(bn.momentum), float(bn.eps), float(act.negative_slope)]
    idx0 = None
    if getattr(ops._tls, "cache", None) is not None:
        # inside a kNN-sharing scope (Net.forward): block 1's kNN is the scope's entry
        idx0 = ops.knn_raw(x, model.k, order=ops.reduction_order(x), out_dtype=torch.int32)
    return torch.ops.dgx_host.dgcnn_train(x, params, bufs, idx0, model.k, hyper)
