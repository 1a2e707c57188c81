"""dgx — MI355X-native EdgeConv engine (HIP kernels in libdgx.so, C ABI in include/dgx.h).

Python surface:
  ops.knn / ops.graph_feature     drop-ins for reference models/dgcnn.py:6-44
  edgeconv.edgeconv_stack         the fused DGCNN block chain (dgcnn.py:84-100)
"""
from . import _native  # noqa: F401
from .ops import knn, graph_feature, reduction_order  # noqa: F401
from .edgeconv import edgeconv_stack  # noqa: F401

__all__ = ["knn", "graph_feature", "reduction_order", "edgeconv_stack"]
