"""compute_hog_1x1's work after the kNN call, on the device (SURVEY §8 row f1;
reference models/model_partseg.py:28-92): one C-ABI call (dgx_hog_1x1_sem_f32,
csrc/hog.hip) replaces the D2H copy, np.linalg.svd over B*N neighbourhoods,
the H2D copy and the histogram votes. No host round trip; host tensors take
the CPU path.

The reference runs its stages on different devices depending on the caller
(model_partseg.py:32 the mean on x's device; :42-47 the votes on the GPU
unless use_cpu without LOCAL_RANK), and torch's CPU and GPU kernels round
differently (scalar division, acos / atan, reduction order). ``mean_device``
/ ``votes_device`` say which of torch's kernels the engine reproduces for each
stage; the default is the reference's path for a GPU cloud in Net.forward
(both on the GPU)."""
import torch

from . import _native as N
from . import cpu

# k range of the device path: csrc/svd3.h restates LAPACK dgesdd's tall-matrix
# path (QR first), which dgesdd takes for k >= 5 rows (its mnthr = 3*11/6), and
# the neighbourhood lives in registers up to 64 rows (HOG_MAX_K)
HOG_K_MIN, HOG_K_MAX = 5, 64


def semantics(mean_device, votes_device):
    """The C ABI's `sem` mask (DGX_HOG_MEAN_DEVICE | DGX_HOG_VOTES_DEVICE)."""
    return int(bool(mean_device)) | 2 * int(bool(votes_device))


def hog_1x1(x, idx, mean_device=True, votes_device=True):
    """x (B, 3, N) fp32 on the device, idx (B, N, k) int64 local kNN ids ->
    (B, N, 18) histograms, as the reference computes them from the same idx
    with its mean on the GPU (``mean_device``) or the host, and its votes on
    the GPU (``votes_device``) or the host. Host tensors take the reference's
    own host path (dgx.cpu.hog_1x1)."""
    if torch.compiler.is_compiling():   # traced as one dgx::hog_1x1 op (dgx.library)
        from . import library  # noqa: F401
        return torch.ops.dgx.hog_1x1(x, idx)
    if cpu.is_cpu(x) and cpu.is_cpu(idx):
        return cpu.hog_1x1(x, idx)
    N.require_device(x, idx)
    B, C, P = x.shape
    if C != 3:
        raise RuntimeError(f"dgx: compute_hog_1x1 takes (B, 3, N) clouds, got {tuple(x.shape)}")
    k = idx.shape[-1]
    if not HOG_K_MIN <= k <= HOG_K_MAX:
        raise NotImplementedError(f"dgx: compute_hog_1x1 on the device supports {HOG_K_MIN} <= k <= {HOG_K_MAX} "
                                  f"neighbours (got k={k}); the reference's numpy SVD path takes any k")
    if tuple(idx.shape) != (B, P, k):
        raise RuntimeError(f"dgx: kNN ids of shape {tuple(idx.shape)} do not match the cloud {tuple(x.shape)}")
    x = x.contiguous()
    idx = idx.contiguous()
    axis = torch.empty((P, 4), device=x.device, dtype=torch.float32)
    out = torch.empty((B, P, 18), device=x.device, dtype=torch.float32)
    N.check(N.lib().dgx_hog_1x1_sem_f32(N.f32(x), N.ptr(idx, N.I64), B, P, k, semantics(mean_device, votes_device),
                                        N.f32(axis), N.f32(out), N.stream_of(x)), "hog_1x1")
    return out
