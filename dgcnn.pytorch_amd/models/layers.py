"""Drop-in for reference ``models/layers.py``: ``PositionEmbedding``.

Reference layers.py:8-74 — a spatial-transform block: edge features of the
input cloud (layers.py:45, via ``get_graph_feature`` bound by name from
models.dgcnn, as the reference does at layers.py:6), two per-edge 1x1 convs
with BN + LeakyReLU, max over k, a per-point 128->1024 conv, max over points,
an MLP to a 3x3 matrix (identity-initialised) and ``bmm`` with the input.
Parameter and buffer names match the reference, including the ``bn1/bn2/bn3``
aliases of ``conv{1,2,3}.1``.
"""
import torch
import torch.nn as nn
import torch.nn.init as init

from models.dgcnn import get_graph_feature


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
        edges = get_graph_feature(x, k=self.k)                   # (B, 6, N, k)    layers.py:45
        t = self.conv2(self.conv1(edges)).max(dim=-1)[0]          # (B, 128, N)     layers.py:48-52
        t = self.conv3(t).max(dim=-1)[0]                          # (B, 1024)       layers.py:55-57
        t = self.transform(self.linear(t)).view(n_clouds, 3, 3)   # (B, 3, 3)       layers.py:60-65
        return torch.bmm(x.transpose(2, 1), t).transpose(2, 1)    # (B, 3, N)       layers.py:68-72
