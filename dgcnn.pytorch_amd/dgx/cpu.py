"""CPU dispatch of the engine's building blocks ("CPU tensors ->
CPU restatement path").

The reference runs its hot path on CPU tensors too (models/dgcnn.py:19-20
picks the device from the input; BASELINE cfg1 is main_cls.py at B=4 on the
host). Every engine entry point — ``knn``, ``graph_feature``, the EdgeConv
block chain, the point conv, the PositionEmbedding edge stage, the HOG
histogram and the attention — sends a CPU tensor here and a ROCm tensor to
libdgx.so; a ROCm tensor never reaches this module (no fallback: a missing
HIP library still raises on the device path).

The arithmetic is torch's CPU kernels, so results follow the reference:
  * ``knn``: the reference's own op sequence (dgcnn.py:7-11: matmul, sum of
    squares, the two broadcast subtractions), bit for bit the same values; the
    top-k is a stable descending sort, i.e. ties in canonical (index
    ascending) order, as on the device (the reference's topk orders ties
    arbitrarily).
  * EdgeConv blocks: the decomposition the device uses — the 1x1 conv on
    cat(x_j, x_i) is P_j + Q_i with P = X W1^T, Q = X W2^T (dgcnn.py:41-43, 55)
    — then the block's own BatchNorm / LeakyReLU modules and the max over k,
    with torch autograd. k times fewer GEMM flops than the edge tensor; equal
    to the reference within fp32 rounding (the 1e-3 parity bar).
  * the other stages call the reference modules on the same tensors.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def is_cpu(t):
    return isinstance(t, torch.Tensor) and t.device.type == "cpu"


def knn(x, k):
    """int64 (B, N, k) local ids (reference dgcnn.py:6-12), canonical tie order."""
    x = x.detach()
    if x.dtype != torch.float32:
        x = x.float()   # distances in fp32 whatever the input
    B, C, N = x.shape
    if not (1 <= k <= N):
        raise RuntimeError(f"knn: selected index k out of range (k={k}, N={N})")
    inner = -2 * torch.matmul(x.transpose(2, 1).contiguous(), x)
    xx = torch.sum(x ** 2, dim=1, keepdim=True)
    pd = -xx - inner - xx.transpose(2, 1).contiguous()
    return pd.sort(dim=-1, descending=True, stable=True)[1][..., :k].contiguous()


def graph_feature(x, k=20, knn_only=False, disp_only=False, idx=None, mode="cat"):
    """Edge features of reference dgcnn.py:15-44 (differentiable in x);
    mode "diff": (x_j - x_i, x_i) of test.ipynb:131."""
    if x.dtype != torch.float32:
        x = x.float()
    B, C, N = x.shape
    if idx is None:
        idx = knn(x, k)
    k = idx.shape[-1]
    flat = (idx.long() + torch.arange(B).view(-1, 1, 1) * N).view(-1)
    rows = x.transpose(2, 1).contiguous()
    nbr = rows.view(B * N, -1)[flat, :].view(B, N, k, C)
    if knn_only:
        return nbr
    ctr = rows.view(B, N, 1, C).repeat(1, 1, k, 1)
    if disp_only:
        return (nbr - ctr).permute(0, 3, 1, 2).contiguous()
    first = nbr - ctr if mode == "diff" else nbr
    return torch.cat((first, ctr), dim=3).permute(0, 3, 1, 2).contiguous()


def _edge_values(x, idx, weight):
    """y[b, o, i, j] = (W [x_j; x_i])_o for the kNN edges (i, idx[i, j]) of
    every cloud, as P_j + Q_i (B, Co, N, k)."""
    B, C, N = x.shape
    k = idx.shape[-1]
    Co = weight.shape[0]
    w = weight.reshape(Co, 2 * C)
    rows = x.transpose(2, 1)                                        # (B, N, C)
    P = torch.matmul(rows, w[:, :C].t())                            # (B, N, Co)
    Q = torch.matmul(rows, w[:, C:].t())
    flat = (idx.long() + torch.arange(B).view(-1, 1, 1) * N).view(-1)
    Pj = P.reshape(B * N, Co)[flat].view(B, N, k, Co)
    return (Pj + Q.unsqueeze(2)).permute(0, 3, 1, 2)               # (B, Co, N, k)


def edgeconv_block(x, k, seq, weight=None):
    """max_k LeakyReLU(BN(Conv2d_1x1(get_graph_feature(x, k)))), reference
    dgcnn.py:84-98, with the block's own modules; x (B, C, N) -> (B, Co, N).
    ``weight``: the conv weight to use instead of the module's (edge_mode "diff")."""
    conv, bn, act = seq[0], seq[1], seq[2]
    y = _edge_values(x, knn(x, k), conv.weight if weight is None else weight)
    if conv.bias is not None:
        y = y + conv.bias.view(1, -1, 1, 1)
    return act(bn(y)).max(dim=-1, keepdim=False)[0]


def edgeconv_stack_pair(x, k, convs, training=None, preps=None, weights=None):
    """The engine's chain contract (dgx.edgeconv.edgeconv_stack_pair): the
    blocks' outputs concatenated point-major (B*N, sum Co), and an empty bf16
    twin. Block l > 1 searches its neighbours on the previous block's
    contiguous (B, C, N) output, as the reference does (dgcnn.py:86-96)."""
    if x.dtype != torch.float32:
        x = x.float()
    B, _, N = x.shape
    h, outs = x, []
    for li, seq in enumerate(convs):
        h = edgeconv_block(h, k, seq, None if weights is None else weights[li])
        outs.append(h)
    cat = torch.cat(outs, dim=1)                                    # (B, sum Co, N)  dgcnn.py:100
    return cat.permute(0, 2, 1).reshape(B * N, -1), torch.empty(0, dtype=torch.bfloat16)


def pointconv_bn_lrelu(X, B, N, seq, training=None, X16=None, wprep=None):
    """X (B*N, K) point-major -> (B, Co, N) = seq(X) with the modules of seq
    (reference dgcnn.py:100-102: conv5 on the unsqueezed concat)."""
    K = X.shape[1]
    z = X.view(B, N, K).permute(0, 2, 1)
    if isinstance(seq[0], torch.nn.Conv2d):
        return seq(z.unsqueeze(-1)).view(B, -1, N)
    return seq(z)


def edge_mlp2(x, k, conv1, conv2, training=None, knn_src=None):
    """max_k conv2(conv1(get_graph_feature(x, k))) (reference layers.py:45-52):
    conv1 decomposed over the kNN graph, conv2 on the (B, C1, N, k) edges."""
    if x.dtype != torch.float32:
        x = x.float()
    idx = knn(knn_src if knn_src is not None else x, k)
    c1, bn1, a1 = conv1[0], conv1[1], conv1[2]
    y1 = _edge_values(x, idx, c1.weight)
    h1 = a1(bn1(y1))
    return conv2(h1).max(dim=-1, keepdim=False)[0].contiguous()


def hog_1x1(x, idx):
    """compute_hog_1x1 after its kNN call (reference model_partseg.py:28-92) on
    the host, as the reference runs it: LAPACK SVD (numpy) of every point's
    centred neighbourhood, the first right singular vector's angles voted into
    9 bins of 20 degrees per angle, L2-normalised. The neighbourhood gather uses
    LOCAL ids over x.view(B*N, -1), as the reference does."""
    B, _, P = x.shape
    k = idx.shape[-1]
    nn_idx = idx.reshape(-1)
    x_nn = x.contiguous().view(B * P, -1)[nn_idx, :].view(B, P, k, 3)
    centered = x_nn - x_nn.mean(dim=2, keepdim=True)
    _, s, v = np.linalg.svd(centered.detach().numpy(), full_matrices=False)
    v = torch.from_numpy(v)
    s = torch.from_numpy(np.sqrt(s))
    grad = v[:, :, 0].reshape(B * P, -1)[nn_idx, :].view(B, P, k, 3)
    mag = s[:, :, 0].unsqueeze(-1).reshape(B * P, -1)[nn_idx, :].view(B, P, k, 1)
    zenith = torch.acos(grad[..., 2]).unsqueeze(-1) * 180 / np.pi
    azimuth = torch.atan(grad[..., 1] / grad[..., 0]).unsqueeze(-1) * 180 / np.pi
    cells = torch.cat((zenith.int(), azimuth.int(), mag), dim=-1)
    cells[cells < 0] += 180
    hist = torch.zeros((B, P, 9, 2))
    bins = torch.floor(cells[..., :2] / 20.0 - 0.5) % 9
    first = cells[..., 2].unsqueeze(-1) * ((20.0 * ((bins + 1) % 9 + 0.5) - cells[..., :2]) % 180) / 20.0
    second = cells[..., 2].unsqueeze(-1) * ((cells[..., :2] - 20.0 * (bins + 0.5)) % 180) / 20.0
    for c in range(9):
        hist[:, :, c] += (first * (bins == c)).sum(dim=2)
        hist[:, :, (c + 1) % 9] += (second * (bins == c)).sum(dim=2)
    return F.normalize(hist, p=2.0, dim=2).view(B, P, -1)


def attention(q, k, v, heads, dropout_p=0.0, scale=None):
    """dropout(softmax(scale q k^T)) v per head on the host (torch's
    scaled_dot_product_attention, the kernel nn.MultiheadAttention uses)."""
    B, Nq, E = q.shape
    D = E // heads
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    qh, kh, vh = (t.reshape(B, -1, heads, D).transpose(1, 2) for t in (q, k, v))
    o = F.scaled_dot_product_attention(qh, kh, vh, dropout_p=dropout_p, scale=scale)
    return o.transpose(1, 2).reshape(B, Nq, E)

