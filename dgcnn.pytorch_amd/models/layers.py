"""Drop-in for reference ``models/layers.py``: ``PositionEmbedding``.

Reference layers.py:8-74 — a spatial-transform block: edge features of the
input cloud (layers.py:45, via ``get_graph_feature`` bound by name from
models.dgcnn, as the reference does at layers.py:6), two per-edge 1x1 convs
with BN + LeakyReLU, max over k, a per-point 128->1024 conv, max over points,
an MLP to a 3x3 matrix (identity-initialised) and ``bmm`` with the input.
Parameter and buffer names match the reference, including the ``bn1/bn2/bn3``
aliases of ``conv{1,2,3}.1``.

The edge stage (layers.py:45-52: graph feature -> conv1 -> conv2 -> max over
k) runs as one engine op, ``dgx.edgemlp.edge_mlp2``: conv1 decomposed over the
kNN graph (the (B,6,N,k) edge tensor is never built), conv2 as an MFMA GEMM
over the B*N*k edge rows, BN statistics, LeakyReLU and the max fused into HIP
kernels (csrc/edgemlp.hip).
"""
import torch
import torch.nn as nn
import torch.nn.init as init

from dgx.edgemlp import edge_mlp2
from models.dgcnn import get_graph_feature  # noqa: F401  (bound by name as at layers.py:6)


def _lrelu(inplace=False):
    return nn.LeakyReLU(negative_slope=0.2, inplace=inplace)


class PositionEmbedding(nn.Module):
    '''Adapted from Transform Block of DGCNN'''

    def __init__(self, args):
        super().__init__()
        self.k = args.k
        self.bn1, self.bn2, self.bn3 = nn.BatchNorm2d(64), nn.BatchNorm2d(128), nn.BatchNorm1d(1024)
        self.conv1 = nn.Sequential(nn.Conv2d(6, 64, kernel_size=1, bias=False), self.bn1, _lrelu())
        self.conv2 = nn.Sequential(nn.Conv2d(64, 128, kernel_size=1, bias=False), self.bn2, _lrelu())
        self.conv3 = nn.Sequential(nn.Conv1d(128, 1024, kernel_size=1, bias=False), self.bn3, _lrelu())
        mlp = []
        for c_in, c_out in ((1024, 512), (512, 256)):
            mlp += [nn.Linear(c_in, c_out, bias=False), nn.BatchNorm1d(c_out), _lrelu(inplace=True)]
        self.linear = nn.Sequential(*mlp)
        self.transform = nn.Linear(256, 9)
        init.constant_(self.transform.weight, 0)
        init.eye_(self.transform.bias.view(3, 3))

    def forward(self, x):
        n_clouds = x.size(0)
        # get_graph_feature + conv1 + conv2 + max over k, fused   (B, 128, N)     layers.py:45-52
        t = edge_mlp2(x, self.k, self.conv1, self.conv2, self.training)
        t = self.conv3(t).max(dim=-1)[0]                          # (B, 1024)       layers.py:55-57
        t = self.transform(self.linear(t)).view(n_clouds, 3, 3)   # (B, 3, 3)       layers.py:60-65
        return torch.bmm(x.transpose(2, 1), t).transpose(2, 1)    # (B, 3, N)       layers.py:68-72
