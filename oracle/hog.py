"""TEST INFRASTRUCTURE ONLY — torch-CPU restatement of the reference's
compute_hog_1x1 after its kNN call (models/model_partseg.py:28-92), given the
kNN ids. The checker for dgx_hog_1x1_f32 (csrc/hog.hip); pinned bit-exactly
by tests/golden/partseg_small.npz (the reference run on CPU, make_goldens.py)
in tests/test_partseg.py."""
import numpy as np
import torch
import torch.nn.functional as F


def hog_1x1(x, idx):
    """x (B,3,N) fp32 CPU tensor, idx (B,N,k) int64 local ids -> (B,N,18)."""
    B, N = x.size(0), x.size(2)
    k = idx.shape[-1]
    flat = torch.as_tensor(idx).reshape(-1)
    # :28-30 local-id gather over the (B*N, 3) view
    x_nn = x.contiguous().view(B * N, -1)[flat, :].view(B, N, k, 3)
    centered = x_nn - x_nn.mean(dim=2, keepdim=True)                       # :32-33
    _, s, v = np.linalg.svd(centered.numpy(), full_matrices=False)         # :36-37
    v = torch.from_numpy(v)
    s = torch.from_numpy(np.sqrt(s))                                      # :40
    gradients = v[:, :, 0]                                                # :49-50
    magnitudes = s[:, :, 0].unsqueeze(-1)
    g = gradients.reshape(B * N, -1)[flat, :].view(B, N, k, 3)            # :53-56
    m = magnitudes.reshape(B * N, -1)[flat, :].view(B, N, k, 1)
    zenith = torch.acos(g[:, :, :, 2]).unsqueeze(-1) * 180 / np.pi       # :58-60
    azimuth = torch.atan(g[:, :, :, 1] / g[:, :, :, 0]).unsqueeze(-1) * 180 / np.pi
    cells = torch.cat((zenith.int(), azimuth.int(), m), dim=-1)          # :62
    cells[cells < 0] += 180                                               # :64
    hist = torch.zeros((B, N, 9, 2))
    bins = torch.floor(cells[:, :, :, :2] / 20.0 - 0.5) % 9              # :76
    first_centers = 20.0 * ((bins + 1) % 9 + 0.5)                         # :80-86
    first_votes = cells[:, :, :, 2].unsqueeze(-1) * ((first_centers - cells[:, :, :, :2]) % 180) / 20.0
    second_centers = 20.0 * (bins + 0.5)
    second_votes = cells[:, :, :, 2].unsqueeze(-1) * ((cells[:, :, :, :2] - second_centers) % 180) / 20.0
    for c in range(9):                                                    # :87-89
        hist[:, :, c] += (first_votes * (bins == c)).sum(dim=2)
        hist[:, :, (c + 1) % 9] += (second_votes * (bins == c)).sum(dim=2)
    return F.normalize(hist, p=2.0, dim=2).view(B, N, -1)                # :90-91
