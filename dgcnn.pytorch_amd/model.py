"""The ``model`` module the reference's scripts import but do not ship
(main_cls.py:25 ``from model import PointNet, DGCNN_cls``, main_semseg.py:20
``from model import DGCNN_semseg``): their EdgeConv blocks run on
the engine.

ARCHITECTURE UNPINNED: the reference contains no definition of these classes,
so nothing fixes their layers or outputs. They follow upstream dgcnn.pytorch's
published layer lists (layer names, widths, pooling and heads as upstream
names them, so its checkpoints' keys match), with one deliberate difference:
the edge feature is this fork's (x_j || x_i) (models/dgcnn.py:42), as every
model of the fork builds it, not upstream's (x_j - x_i || x_i). Parity tests
(tests/test_model_gpu.py) compare them with the same layer list run as stock
PyTorch ops on the same weights.

  PointNet      per-point MLP + max pool + head (no graph; stock torch)
  DGCNN_cls     4 EdgeConv blocks (dgx.edgeconv) + conv5 (dgx.pointconv) +
                max/avg pool + MLP head (main_cls.py:56)
  DGCNN_semseg  S3DIS 9-channel input: 2-conv EdgeConv blocks (dgx.edgemlp) with
                the first graph built on the normalised xyz channels 6:9,
                a 1-conv block, conv6 (dgx.pointconv), global max, per-point
                head to 13 classes (main_semseg.py:155)
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from dgx.edgeconv import edgeconv_stack_pair
from dgx.edgemlp import edge_mlp2
from dgx.pointconv import pointconv_bn_lrelu


def _lrelu():
    return nn.LeakyReLU(negative_slope=0.2)


class PointNet(nn.Module):
    def __init__(self, args, output_channels=40):
        super().__init__()
        self.args = args
        widths = (64, 64, 64, 128, args.emb_dims)
        c = 3
        for i, w in enumerate(widths, start=1):
            setattr(self, f"conv{i}", nn.Conv1d(c, w, kernel_size=1, bias=False))
            setattr(self, f"bn{i}", nn.BatchNorm1d(w))
            c = w
        self.linear1 = nn.Linear(args.emb_dims, 512, bias=False)
        self.bn6 = nn.BatchNorm1d(512)
        self.dp1 = nn.Dropout()
        self.linear2 = nn.Linear(512, output_channels)

    def forward(self, x):
        for i in range(1, 6):
            x = F.relu(getattr(self, f"bn{i}")(getattr(self, f"conv{i}")(x)))
        x = F.adaptive_max_pool1d(x, 1).squeeze(-1)
        x = self.dp1(F.relu(self.bn6(self.linear1(x))))
        return self.linear2(x)


class DGCNN_cls(nn.Module):
    """Classification DGCNN; reads args.k, args.emb_dims, args.dropout."""

    def __init__(self, args, output_channels=40):
        super().__init__()
        self.args = args
        self.k = args.k
        self.bn1, self.bn2, self.bn3, self.bn4 = (nn.BatchNorm2d(64), nn.BatchNorm2d(64), nn.BatchNorm2d(128),
                                                  nn.BatchNorm2d(256))
        self.bn5 = nn.BatchNorm1d(args.emb_dims)
        blocks = ((6, 64, self.bn1), (128, 64, self.bn2), (128, 128, self.bn3), (256, 256, self.bn4))
        for i, (ci, co, bn) in enumerate(blocks, start=1):
            setattr(self, f"conv{i}", nn.Sequential(nn.Conv2d(ci, co, kernel_size=1, bias=False), bn, _lrelu()))
        self.conv5 = nn.Sequential(nn.Conv1d(512, args.emb_dims, kernel_size=1, bias=False), self.bn5, _lrelu())
        self.linear1 = nn.Linear(args.emb_dims * 2, 512, bias=False)
        self.bn6 = nn.BatchNorm1d(512)
        self.dp1 = nn.Dropout(p=args.dropout)
        self.linear2 = nn.Linear(512, 256)
        self.bn7 = nn.BatchNorm1d(256)
        self.dp2 = nn.Dropout(p=args.dropout)
        self.linear3 = nn.Linear(256, output_channels)

    def forward(self, x):
        B, _, N = x.shape
        feats, feats16 = edgeconv_stack_pair(x, self.k, [self.conv1, self.conv2, self.conv3, self.conv4])
        x = pointconv_bn_lrelu(feats, B, N, self.conv5, X16=feats16)          # (B, emb, N)
        x = torch.cat((F.adaptive_max_pool1d(x, 1).view(B, -1), F.adaptive_avg_pool1d(x, 1).view(B, -1)), 1)
        x = self.dp1(F.leaky_relu(self.bn6(self.linear1(x)), negative_slope=0.2))
        x = self.dp2(F.leaky_relu(self.bn7(self.linear2(x)), negative_slope=0.2))
        return self.linear3(x)


class DGCNN_semseg(nn.Module):
    """Semantic segmentation DGCNN on (B, 9, N) S3DIS blocks; reads args.k,
    args.emb_dims, args.dropout. Output (B, 13, N)."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        self.k = args.k
        for i, w in enumerate((64, 64, 64, 64, 64), start=1):
            setattr(self, f"bn{i}", nn.BatchNorm2d(w))
        self.bn6 = nn.BatchNorm1d(args.emb_dims)
        self.bn7 = nn.BatchNorm1d(512)
        self.bn8 = nn.BatchNorm1d(256)
        pairs = ((18, 64), (64, 64), (128, 64), (64, 64), (128, 64))
        for i, (ci, co) in enumerate(pairs, start=1):
            setattr(self, f"conv{i}", nn.Sequential(nn.Conv2d(ci, co, kernel_size=1, bias=False),
                                                    getattr(self, f"bn{i}"), _lrelu()))
        self.conv6 = nn.Sequential(nn.Conv1d(192, args.emb_dims, kernel_size=1, bias=False), self.bn6, _lrelu())
        self.conv7 = nn.Sequential(nn.Conv1d(args.emb_dims + 192, 512, kernel_size=1, bias=False), self.bn7,
                                   _lrelu())  # 1216 at the default emb_dims 1024
        self.conv8 = nn.Sequential(nn.Conv1d(512, 256, kernel_size=1, bias=False), self.bn8, _lrelu())
        self.dp1 = nn.Dropout(p=args.dropout)
        self.conv9 = nn.Conv1d(256, 13, kernel_size=1, bias=False)

    def forward(self, x):
        B, _, N = x.shape
        # block 1: graph on the normalised xyz channels 6:9, edge features of all 9
        x1 = edge_mlp2(x, self.k, self.conv1, self.conv2, knn_src=x[:, 6:9])          # (B, 64, N)
        x2 = edge_mlp2(x1.contiguous(), self.k, self.conv3, self.conv4)             # (B, 64, N)
        x3, _ = edgeconv_stack_pair(x2.contiguous(), self.k, [self.conv5])        # (B*N, 64)
        x3 = x3.view(B, N, -1).permute(0, 2, 1)
        pm = torch.cat([t.permute(0, 2, 1).reshape(B * N, -1) for t in (x1, x2, x3)], dim=1)
        g = pointconv_bn_lrelu(pm, B, N, self.conv6).max(dim=-1, keepdim=True)[0]  # (B, emb, 1)
        x = torch.cat((g.repeat(1, 1, N), x1, x2, x3), dim=1)
        x = self.dp1(self.conv8(self.conv7(x)))
        return self.conv9(x)
