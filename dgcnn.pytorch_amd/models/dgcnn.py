"""Drop-in for reference ``models/dgcnn.py``: ``knn``, ``get_graph_feature``, ``DGCNN``.

Same names, signatures, defaults, return shapes/dtypes and ``state_dict`` keys
as the reference (models/dgcnn.py:6-103), so ``from models.dgcnn import ...``
sites (models/layers.py:6, models/model_partseg.py:11) bind to this module
unchanged. The work runs in libdgx.so on the MI355X:

* ``knn``  -> fused fp32 distance + top-k kernel, bit-exact distances, ties in
  canonical order (the reference's CPU ``topk`` order for ties is arbitrary).
* ``get_graph_feature`` -> gather kernel writing the reference's layout.
* ``DGCNN.forward`` never materialises the (B,2C,N,k) edge tensors: the four
  EdgeConv blocks run as one fused chain (dgx.edgeconv), conv5 is a GEMM on
  the concat buffer the chain writes in place (dgx.pointconv).
"""
import torch
import torch.nn as nn

from dgx import host as _host
from dgx import library as _library
from dgx import ops as _ops
from dgx.edgeconv import edgeconv_stack_pair
from dgx.pointconv import pointconv_bn_lrelu


def knn(x, k):
    """(B,C,N) -> int64 (B,N,k) local indices of the k largest
    ``-|x_i - x_j|^2`` per point (self included), reference dgcnn.py:6-12."""
    return _ops.knn(x, k)


def get_graph_feature(x, k=20, knn_only=False, disp_only=False, mode="cat"):
    """Edge features of reference dgcnn.py:15-44 (differentiable in x).
    ``mode="diff"`` (engine extension) gives the paper's (x_j - x_i, x_i)
    form of test.ipynb:131 instead of dgcnn.py:42's (x_j, x_i)."""
    return _ops.graph_feature(x, k=k, knn_only=knn_only, disp_only=disp_only, mode=mode)


def _edge_block(c_in, c_out):
    # Conv2d(2C, Co, 1, bias=False) -> BatchNorm2d -> LeakyReLU(0.2), dgcnn.py:54-73
    return nn.Sequential(nn.Conv2d(2 * c_in, c_out, kernel_size=1, bias=False),
                         nn.BatchNorm2d(c_out),
                         nn.LeakyReLU(negative_slope=0.2, inplace=True))


def _diff_weight(w):
    """The conv weight that applied to (x_j, x_i) equals ``w`` applied to
    (x_j - x_i, x_i): [W1 | W2] -> [W1 | W2 - W1] (differentiable, so the
    module's gradient follows by autograd)."""
    c = w.shape[1] // 2
    return torch.cat([w[:, :c], w[:, c:] - w[:, :c]], dim=1)


class DGCNN(nn.Module):
    """4 EdgeConv blocks (3->64->64->128->256) + conv5 (512->emb); input
    (B,3,N), output (B,emb,N). Reads ``args.emb_dim`` and ``args.k``
    (reference dgcnn.py:47-78). Engine extensions: an optional ``args.in_dims``
    (default 3, the reference's) sets the input channels, e.g. 9 for the S3DIS
    block layout (prepare_data/indoor3d_util.py:238-261); an optional
    ``args.edge_mode`` "diff" makes each block see the paper's edge feature
    (x_j - x_i, x_i) (test.ipynb:131) instead of dgcnn.py:42's (x_j, x_i) — the
    same kernels on the re-parameterised weight [W1 | W2 - W1]. The default
    model's parameters and state_dict are the reference's."""

    WIDTHS = (64, 64, 128, 256)

    def __init__(self, args):
        super().__init__()
        self.emb_dims = args.emb_dim
        self.k = args.k
        self.edge_mode = getattr(args, "edge_mode", "cat")
        if self.edge_mode not in ("cat", "diff"):
            raise ValueError(f"DGCNN: edge_mode must be 'cat' or 'diff', got {self.edge_mode!r}")
        c_in = getattr(args, "in_dims", 3)
        for i, c_out in enumerate(self.WIDTHS, start=1):
            setattr(self, f"conv{i}", _edge_block(c_in, c_out))
            c_in = c_out
        self.conv5 = nn.Sequential(nn.Conv2d(sum(self.WIDTHS), self.emb_dims, kernel_size=1, bias=False),
                                   nn.BatchNorm2d(self.emb_dims),
                                   nn.LeakyReLU(negative_slope=0.2, inplace=True))

    def edge_blocks(self):
        return [self.conv1, self.conv2, self.conv3, self.conv4]

    def edge_weights(self):
        """The blocks' conv weights as the engine applies them to (x_j, x_i)."""
        ws = [b[0].weight for b in self.edge_blocks()]
        return [_diff_weight(w) for w in ws] if self.edge_mode == "diff" else ws

    def forward(self, x):
        if x.device.type == "cpu":
            # host tensors (reference dgcnn.py:19-20 runs on either device): the
            # CPU path of every block (dgx.cpu), same modules and state
            feats, _ = edgeconv_stack_pair(x, self.k, self.edge_blocks(), self.training, weights=self.edge_weights())
            return pointconv_bn_lrelu(feats, x.shape[0], x.shape[2], self.conv5, self.training)
        if torch.compiler.is_compiling() and _library.enabled_for(self):
            # the same schedule behind torch.ops.dgx custom ops (torch.compile / export see one node each)
            return _library.dgcnn_forward(self, x)
        if _host.applies(self, x):
            # one C++ op + C++ autograd node (libdgx_torch.so), every precision / BN mode
            return _host.dgcnn_forward(self, x)
        batch_size, _, num_points = x.size()
        # the autograd Functions over the same C++ schedule (debug capture, DGX_HOST_EXT=0):
        # x1..x4 of dgcnn.py:84-98, already concatenated point-major (dgcnn.py:100)
        feats, feats16 = edgeconv_stack_pair(x, self.k, self.edge_blocks(), self.training,
                                             weights=self.edge_weights())   # (B*N, 512)
        # conv5 -> BN -> LeakyReLU (dgcnn.py:100-102), written as (B, emb, N)
        return pointconv_bn_lrelu(feats, batch_size, num_points, self.conv5, self.training, X16=feats16)
