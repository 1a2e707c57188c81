"""TEST INFRASTRUCTURE ONLY — torch-CPU restatement of the reference's float path.

Used by tests/ (1e-3 parity of the HIP path) and by bench.py's cpu_baseline
leg (the reference's CPU path timed on the GPU box's host cores: the reference
source cannot travel, this restatement does, and tests/golden pins it to the
reference's own outputs). Never imported by the product.

Functional restatement of reference models/dgcnn.py:6-103 and
models/layers.py:8-74 using the same ATen ops (matmul, sum, topk, index,
repeat, cat, permute, conv2d, batch_norm, leaky_relu, max).
"""
import torch
import torch.nn.functional as F


def knn(x, k):
    """reference dgcnn.py:6-12 op for op (matmul -> sum -> broadcast subtract -> topk)."""
    gram = torch.matmul(x.transpose(2, 1).contiguous(), x)
    sq = torch.sum(x ** 2, dim=1, keepdim=True)
    neg_d2 = -sq - (-2 * gram) - sq.transpose(2, 1).contiguous()
    return neg_d2.topk(k=k, dim=-1)[1]


def graph_feature(x, k=20, knn_only=False, disp_only=False, idx=None):
    """reference dgcnn.py:15-44; `idx` lets a test inject the neighbour sets."""
    B, C, N = x.shape
    if idx is None:
        idx = knn(x, k)
    k = idx.shape[-1]
    flat = (idx + torch.arange(B, device=x.device).view(-1, 1, 1) * N).reshape(-1)
    rows = x.transpose(2, 1).contiguous()
    nbr = rows.reshape(B * N, C)[flat, :].view(B, N, k, C)
    if knn_only:
        return nbr
    ctr = rows.view(B, N, 1, C).repeat(1, 1, k, 1)
    if disp_only:
        return (nbr - ctr).permute(0, 3, 1, 2).contiguous()
    return torch.cat((nbr, ctr), dim=3).permute(0, 3, 1, 2).contiguous()


def conv_bn_lrelu(x, weight, bn, training, slope=0.2):
    """Conv(1x1, no bias) -> BatchNorm (train or eval) -> LeakyReLU.
    bn: dict with weight, bias, running_mean, running_var (updated in place when
    training), momentum, eps."""
    if x.dim() == 4:
        y = F.conv2d(x, weight)
    else:
        y = F.conv1d(x, weight)
    y = F.batch_norm(y, bn["running_mean"], bn["running_var"], bn["weight"], bn["bias"], training,
                     bn.get("momentum", 0.1), bn.get("eps", 1e-5))
    return F.leaky_relu(y, slope)


def edgeconv_block(x, k, weight, bn, training, idx=None, slope=0.2):
    """One DGCNN block (dgcnn.py:84-86): graph feature -> conv/BN/LReLU -> max_k."""
    e = graph_feature(x, k, idx=idx)
    return conv_bn_lrelu(e, weight, bn, training, slope).max(dim=-1, keepdim=False)[0]


def dgcnn(x, k, params, training, idx_list=None):
    """reference DGCNN.forward (dgcnn.py:80-103). params: dict name -> tensor
    laid out like DGCNN.state_dict() (conv{i}.0.weight, conv{i}.1.*).
    idx_list: optional per-block neighbour indices to inject (else computed)."""
    B, _, N = x.shape
    feats, h, used = [], x, []
    for i in range(1, 5):
        bn = _bn(params, f"conv{i}.1")
        idx = None if idx_list is None else idx_list[i - 1]
        if idx is None:
            idx = knn(h, k)
        used.append(idx)
        h = edgeconv_block(h, k, params[f"conv{i}.0.weight"], bn, training, idx=idx)
        feats.append(h)
    z = torch.cat(feats, dim=1).unsqueeze(-1)
    z = conv_bn_lrelu(z, params["conv5.0.weight"], _bn(params, "conv5.1"), training)
    return z.view(B, -1, N), used


def _bn(params, prefix):
    return {"weight": params[prefix + ".weight"], "bias": params[prefix + ".bias"],
            "running_mean": params[prefix + ".running_mean"], "running_var": params[prefix + ".running_var"],
            "momentum": 0.1, "eps": 1e-5}


# --------------------------------------------------------------------------
# Decision-routed variants. max_k and LeakyReLU are non-smooth: at a near-tie
# of the max or at z ~ 0, any change of fp32 summation order (GPU vs CPU, or
# the engine's P_j + Q_i decomposition) can route a gradient differently. To
# hold gradients to 1e-3 the oracle below re-uses the engine's DECISIONS (the
# selected neighbour per (point, channel) and the sign of the selected BN
# output) and recomputes everything else in fp64. The tests separately check
# that each decision is valid (the chosen edge is a max up to rounding; a sign
# only differs where |z| is at rounding level).

def edgeconv_block_routed(x, weight, bn, idx, arg, zpos, slope=0.2, training=True):
    """x (B,C,N); idx (B,N,k); arg (B*N,Co) chosen k-slot; zpos (B*N,Co) bool.
    training=False normalises with the running statistics (BatchNorm eval)."""
    e = graph_feature(x, idx=idx)
    y = F.conv2d(e, weight)
    z = F.batch_norm(y, bn["running_mean"], bn["running_var"], bn["weight"], bn["bias"], training,
                     bn.get("momentum", 0.1), bn.get("eps", 1e-5))
    B, Co, N, _ = z.shape
    a = arg.long().view(B, N, Co).permute(0, 2, 1).unsqueeze(-1)
    zsel = torch.gather(z, 3, a).squeeze(-1)
    m = zpos.view(B, N, Co).permute(0, 2, 1)
    return torch.where(m, zsel, slope * zsel), z


def dgcnn_routed(x, params, decisions, mask5, slope=0.2, training=(True,) * 5):
    """DGCNN forward with the engine's decisions: decisions[l] = (idx, arg, zpos)
    for blocks 1-4, mask5 (B,emb,N) bool = sign of conv5's BN output.
    training[l]: batch (True) or running (False) statistics for BN l+1."""
    B, _, N = x.shape
    h, feats = x, []
    for i in range(1, 5):
        idx, arg, zpos = decisions[i - 1]
        h, _ = edgeconv_block_routed(h, params[f"conv{i}.0.weight"], _bn(params, f"conv{i}.1"), idx, arg, zpos, slope,
                                     training[i - 1])
        feats.append(h)
    z = torch.cat(feats, dim=1).unsqueeze(-1)
    z = F.conv2d(z, params["conv5.0.weight"])
    bn = _bn(params, "conv5.1")
    z = F.batch_norm(z, bn["running_mean"], bn["running_var"], bn["weight"], bn["bias"], training[4], 0.1, 1e-5)
    z = z.view(B, -1, N)
    return torch.where(mask5, z, slope * z)


def edge_mlp2_routed(x, w1, bn1, w2, bn2, idx, zpos1, arg2, zpos2, slope=0.2, training=(True, True)):
    """PositionEmbedding's edge stage (reference models/layers.py:45-52:
    get_graph_feature -> conv1 -> conv2 -> max over k) in x's dtype, routed by
    the engine's decisions: zpos1 (B,C1,N,k) bool = sign of BN1's output per
    edge (conv1's LeakyReLU), arg2 (B*N,C2) = the selected k-slot of conv2's
    max, zpos2 (B*N,C2) bool = sign of BN2's output there. Returns the stage
    output (B,C2,N) and conv2's BN output z2 (B,C2,N,k)."""
    e = graph_feature(x, idx=idx)
    z1 = F.batch_norm(F.conv2d(e, w1), bn1["running_mean"], bn1["running_var"], bn1["weight"], bn1["bias"],
                      training[0], bn1.get("momentum", 0.1), bn1.get("eps", 1e-5))
    h1 = torch.where(zpos1, z1, slope * z1)
    z2 = F.batch_norm(F.conv2d(h1, w2), bn2["running_mean"], bn2["running_var"], bn2["weight"], bn2["bias"],
                      training[1], bn2.get("momentum", 0.1), bn2.get("eps", 1e-5))
    B, C2, N, _ = z2.shape
    a = arg2.long().view(B, N, C2).permute(0, 2, 1).unsqueeze(-1)
    zsel = torch.gather(z2, 3, a).squeeze(-1)
    m = zpos2.view(B, N, C2).permute(0, 2, 1)
    return torch.where(m, zsel, slope * zsel), z2
