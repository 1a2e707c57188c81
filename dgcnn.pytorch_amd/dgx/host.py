"""Eager dispatch of DGCNN.forward through the C++ op layer (libdgx_torch.so,
csrc/dgx_torch.cpp): ``torch.ops.dgx_host.dgcnn`` runs the EdgeConv chain +
conv5 forward (reference models/dgcnn.py:80-103) and, from a C++ autograd
node, the whole backward — the ~60 launches of a step are issued from C++
instead of one Python dispatch each.

It is the same schedule the engine's autograd Functions (dgx.edgeconv,
dgx.pointconv) and torch.library ops (dgx.library) call, one C++
implementation for every configuration the reference's scripts run:
precision bf16, fp32 or fp32_split (bf16 autocast -> bf16 GEMMs, fp16
autocast -> split-bf16 fp32 GEMMs, dgx.precision.effective), BatchNorm in
training or eval mode, momentum or cumulative running statistics, plain
BatchNorm2d or SyncBatchNorm (main_partseg_dist.py:189: the statistics
all-reduce is issued from C++ over the module's process
group), any (B, C, N, k). The Function path is taken only while tests capture
routing decisions (dgx.edgeconv.set_debug_capture), while torch.compile traces
(dgx.library ops), or with ``DGX_HOST_EXT=0`` (A/B runs).
"""
import os
import threading

import torch

from . import bn as bn_
from . import edgeconv as E
from . import ops
from . import precision as prec

ENABLED = os.environ.get("DGX_HOST_EXT", "1") == "1"
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DGX_TORCH_LIB", os.path.join(_HERE, "libdgx_torch.so"))
_lock = threading.Lock()
_loaded = False


def load():
    """Register torch.ops.dgx_host (once). The engine's device schedule lives
    there: a missing libdgx_torch.so is an error, never a fallback."""
    global _loaded
    if not _loaded:
        with _lock:
            if not _loaded:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(f"dgx: C++ op library not built ({LIB_PATH}); run `make -C "
                                      "dgcnn.pytorch_amd/csrc` or __graft_entry__.build()")
                from . import _native
                _native.lib()   # libdgx.so first: libdgx_torch.so links against it
                torch.ops.load_library(LIB_PATH)
                _loaded = True


def applies(model, x):
    """Whether DGCNN ``model``'s forward on ``x`` takes the one-op C++ path."""
    if not ENABLED or torch.compiler.is_compiling() or E.debug_capture() is not None:
        return False
    if x.device.type != "cuda" or x.dim() != 3 or not x.is_floating_point():
        return False
    for seq in model.edge_blocks() + [model.conv5]:
        conv, bn = seq[0], seq[1]
        if conv.bias is not None or bn.weight is None or conv.weight.dtype != torch.float32:
            return False
    return True


def dgcnn_forward(model, x):
    """DGCNN.forward through torch.ops.dgx_host.dgcnn."""
    load()
    eff = prec.effective()
    bf16 = eff == "bf16"
    if x.dtype != torch.float32:
        x = x.float()
    params, bufs, bn_f, bn_i, groups = [], [], [], [], []
    weights = model.edge_weights() + [model.conv5[0].weight]   # re-parameterised in edge_mode "diff"
    for w, seq in zip(weights, model.edge_blocks() + [model.conv5]):
        bn, act = seq[1], seq[2]
        params += [w, bn.weight, bn.bias]
        t, f, i, g = bn_.op_args(bn)
        bufs += t[:3]          # running statistics updated in place
        bn_f += f + [float(act.negative_slope)]
        bn_i += i
        groups.append(g)
    idx0 = None
    if getattr(ops._tls, "cache", None) is not None:
        # inside a kNN-sharing scope (Net.forward): block 1's kNN is the scope's entry
        idx0 = ops.knn_raw(x.detach(), model.k, order=ops.reduction_order(x), out_dtype=torch.int32)
    return torch.ops.dgx_host.dgcnn(x, params, bufs, bn_f, bn_i, groups, idx0, model.k, bf16,
                                    E.opts(eff == "fp32_split"))
