"""TEST INFRASTRUCTURE ONLY — stock-op restatement of the partseg ``Net``
forward (reference models/model_partseg.py:174-194) for routed parity tests.

``stock_copy(net)`` deep-copies an engine ``Net`` with every attention switched
back to torch's own ``nn.MultiheadAttention`` (same parameters), so the
transformer, final attention, label/HOG embeddings, PositionEmbedding tail and
head are the stock PyTorch modules the reference builds. ``net_routed`` runs the
reference's forward over those modules in their dtype (fp64 in the tests), with
the two engine-owned stages restated by ``oracle.reference`` and routed by the
engine's validated decisions:

* ``emb_nn`` (DGCNN, model_partseg.py:177) -> ``reference.dgcnn_routed``;
* ``pos_mlp``'s edge stage (layers.py:45-52) -> ``reference.edge_mlp2_routed``;
* the HOG histogram (model_partseg.py:179, a piecewise-constant function of the
  cloud computed by numpy in the reference, no gradient) is an input, like the
  neighbour sets;
* ``argmax_n`` optionally routes PositionEmbedding's max over points
  (layers.py:55-57) to the engine run's choice (under fp16 autocast its conv3
  output ties / reorders at fp16 resolution).
"""
import copy

import torch
import torch.nn as nn

from . import reference as R


def stock_copy(net):
    """Deep copy of an engine Net whose attentions are torch's nn.MultiheadAttention."""
    m = copy.deepcopy(net)
    for mod in m.modules():
        if isinstance(mod, nn.MultiheadAttention) and type(mod) is not nn.MultiheadAttention:
            mod.__class__ = nn.MultiheadAttention
    return m


def _bn(mod):
    return {"weight": mod.weight, "bias": mod.bias, "running_mean": mod.running_mean,
            "running_var": mod.running_var, "momentum": mod.momentum, "eps": mod.eps}


def net_routed(net, src, lbl, dgcnn_dec, mask5, emlp_dec, hog, argmax_n=None):
    """reference Net.forward (model_partseg.py:174-194) over ``net`` (a
    ``stock_copy``) with the engine's decisions. dgcnn_dec: [(idx, arg, zpos)]
    per EdgeConv block, mask5: sign of emb_nn's conv5 BN output; emlp_dec:
    (idx, zpos1, arg2, zpos2) of PositionEmbedding's edge stage; hog (B,N,18).
    Returns (output (B,nclasses,N), PositionEmbedding's conv3 output (B,1024,N))."""
    B, _, N = src.shape
    p = dict(net.emb_nn.state_dict(keep_vars=True))
    src_emb = R.dgcnn_routed(src, p, dgcnn_dec, mask5)                       # :177
    tgt_emb = net.grads_emb(hog.transpose(1, 2).contiguous())                # :179-180
    pe = net.pos_mlp[0]
    idx, zpos1, arg2, zpos2 = emlp_dec
    t, _ = R.edge_mlp2_routed(src, pe.conv1[0].weight, _bn(pe.bn1), pe.conv2[0].weight, _bn(pe.bn2), idx, zpos1,
                              arg2, zpos2)                                   # layers.py:45-52
    t3 = pe.conv3(t)                                                         # layers.py:55
    if argmax_n is None:
        t = t3.max(dim=-1)[0]
    else:
        t = torch.gather(t3, 2, argmax_n.unsqueeze(-1)).squeeze(-1)
    t = pe.transform(pe.linear(t)).view(B, 3, 3)                            # layers.py:60-65
    canonical = torch.bmm(src.transpose(2, 1), t).transpose(2, 1)          # layers.py:68-72
    canonical = net.pos_mlp[1:](canonical)                                  # :183
    src_emb = (src_emb + canonical).transpose(1, 2)
    tgt_emb = (tgt_emb + canonical).transpose(1, 2)
    src_p = net.transformer(src_emb, tgt_emb)                               # :187
    tgt_p = net.transformer(tgt_emb, src_emb)                               # :188
    scores, _ = net.attention(query=tgt_p, key=src_p, value=src_p, need_weights=False)   # :190
    return net.head(lbl, scores), t3                                        # :192
