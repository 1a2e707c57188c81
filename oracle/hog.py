"""TEST INFRASTRUCTURE ONLY — restatement of the reference's compute_hog_1x1
after its kNN call (models/model_partseg.py:28-92), given the kNN ids. The
checker for dgx_hog_1x1_f32 / dgx_hog_1x1_sem_f32 (csrc/hog.hip).

The reference runs each stage on a device its caller chooses: the gather and
the neighbourhood mean on x's device (:28-33), the SVD on the host (numpy,
:36-40), and the angle / vote / bin-sum / normalize ops (:49-91) on the device
v and s are moved to (:42-47: the GPU when LOCAL_RANK is set or use_cpu is
False, else the host). ``hog_1x1`` runs that same op sequence with the tensors
on the devices given, so the checker is torch's own kernels on each device:
  * x and vote_device on the host: the reference's use_cpu run on a host
    cloud, pinned bit-exactly by tests/golden/partseg_small.npz (the
    reference run on CPU, make_goldens.py) in tests/test_partseg.py;
  * x on the GPU and vote_device "cuda": the reference's default path for a
    GPU cloud (Net.forward, model_partseg.py:179), torch's HIP kernels."""
import numpy as np
import torch
import torch.nn.functional as F


def hog_1x1(x, idx, vote_device=None):
    """x (B,3,N) fp32 tensor, idx (B,N,k) int64 local ids -> (B,N,18) on
    ``vote_device`` (default: x's device)."""
    B, N = x.size(0), x.size(2)
    k = idx.shape[-1]
    vdev = torch.device(vote_device) if vote_device is not None else x.device
    flat = torch.as_tensor(idx).to(x.device).reshape(-1)
    # :28-30 local-id gather over the (B*N, 3) view
    x_nn = x.contiguous().view(B * N, -1)[flat, :].view(B, N, k, 3)
    centered = x_nn - x_nn.mean(dim=2, keepdim=True)                       # :32-33 (x's device)
    _, s, v = np.linalg.svd(centered.detach().cpu().numpy(), full_matrices=False)   # :36-37
    v = torch.from_numpy(v).to(vdev)                                      # :39-47
    s = torch.from_numpy(np.sqrt(s)).to(vdev)
    flat = flat.to(vdev)
    gradients = v[:, :, 0]                                                # :49-50
    magnitudes = s[:, :, 0].unsqueeze(-1)
    g = gradients.reshape(B * N, -1)[flat, :].view(B, N, k, 3)            # :53-56
    m = magnitudes.reshape(B * N, -1)[flat, :].view(B, N, k, 1)
    zenith = torch.acos(g[:, :, :, 2]).unsqueeze(-1) * 180 / np.pi       # :58-60
    azimuth = torch.atan(g[:, :, :, 1] / g[:, :, :, 0]).unsqueeze(-1) * 180 / np.pi
    cells = torch.cat((zenith.int(), azimuth.int(), m), dim=-1)          # :62
    cells[cells < 0] += 180                                               # :64
    hist = torch.zeros((B, N, 9, 2), device=vdev)
    bins = torch.floor(cells[:, :, :, :2] / 20.0 - 0.5) % 9              # :76
    first_centers = 20.0 * ((bins + 1) % 9 + 0.5)                         # :80-86
    first_votes = cells[:, :, :, 2].unsqueeze(-1) * ((first_centers - cells[:, :, :, :2]) % 180) / 20.0
    second_centers = 20.0 * (bins + 0.5)
    second_votes = cells[:, :, :, 2].unsqueeze(-1) * ((cells[:, :, :, :2] - second_centers) % 180) / 20.0
    for c in range(9):                                                    # :87-89
        hist[:, :, c] += (first_votes * (bins == c)).sum(dim=2)
        hist[:, :, (c + 1) % 9] += (second_votes * (bins == c)).sum(dim=2)
    return F.normalize(hist, p=2.0, dim=2).view(B, N, -1)                # :90-91


def hog_bins(x, idx, vote_device=None):
    """The (zenith, azimuth) cells and bins of every (point, neighbour) the
    reference computes (model_partseg.py:58-76): (B, N, k, 2) float tensors on
    the vote device. Used by the tests to report bin agreement."""
    B, N = x.size(0), x.size(2)
    k = idx.shape[-1]
    vdev = torch.device(vote_device) if vote_device is not None else x.device
    flat = torch.as_tensor(idx).to(x.device).reshape(-1)
    x_nn = x.contiguous().view(B * N, -1)[flat, :].view(B, N, k, 3)
    centered = x_nn - x_nn.mean(dim=2, keepdim=True)
    _, _, v = np.linalg.svd(centered.detach().cpu().numpy(), full_matrices=False)
    g = torch.from_numpy(v).to(vdev)[:, :, 0].reshape(B * N, -1)[flat.to(vdev), :].view(B, N, k, 3)
    zenith = torch.acos(g[:, :, :, 2]).unsqueeze(-1) * 180 / np.pi
    azimuth = torch.atan(g[:, :, :, 1] / g[:, :, :, 0]).unsqueeze(-1) * 180 / np.pi
    cells = torch.cat((zenith.int(), azimuth.int()), dim=-1).float()
    cells[cells < 0] += 180
    return cells, torch.floor(cells / 20.0 - 0.5) % 9
