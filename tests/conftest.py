import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dgcnn.pytorch_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libdgx.so")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden


def rel_err(a, b):
    """normwise relative error max|a-b| / max|b| (the 1e-3 fp32 parity metric)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / den)


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU in this container")
    return torch.device("cuda:0")


def check_decisions(z64, arg, zpos, B, N, tol=1e-5):
    """Each engine decision of one max-over-k block must be valid for the fp64
    recomputation z64 (B,Co,N,k): the chosen slot is a maximum of z over k up to
    ``tol`` of z's scale, and the LeakyReLU sign taken there may only disagree
    with z's sign where |z| is below that level. Returns the worst slot gap and
    the worst sign-flip magnitude (both relative to the scale)."""
    import torch
    z = z64.detach()
    Co = z.shape[1]
    scale = float(z.abs().max())
    zmax = z.max(dim=-1)[0]                                                   # (B,Co,N)
    a = arg.long().to(z.device).view(B, N, Co).permute(0, 2, 1).unsqueeze(-1)
    zsel = torch.gather(z, 3, a).squeeze(-1)
    gap = float((zmax - zsel).max()) / scale
    assert gap <= tol, ("max slot", gap, tol)
    zp = zpos.to(z.device).view(B, N, Co).permute(0, 2, 1)
    bad = zp != (zsel > 0)
    flip = float(zsel[bad].abs().max()) / scale if bad.any() else 0.0
    assert flip <= tol, ("LeakyReLU sign", flip, tol)
    return gap, flip


def validate_dgcnn_decisions(cap, x, k, init, training=(True,) * 4, bf16=False, tol=None):
    """Validate EVERY routing decision of an engine DGCNN forward (debug capture
    ``cap``, dgx.edgeconv.set_debug_capture) against the reference's own rules,
    block by block, from the block's engine-produced input (reference
    models/dgcnn.py:84-98):

    * kNN: block l's neighbour sets equal the oracle's kNN (oracle/knn_oracle.c,
      the bit-exact restatement of dgcnn.py:6-12) of that input — for blocks 2-4
      the xcat slice read as (B, C, N) in the reference's strided sum order
      (their input is the contiguous output of a max, dgcnn.py:86-94);
    * max slot and LeakyReLU sign: check_decisions against z recomputed in fp64
      from the same input (graph feature -> conv -> BN with this block's flags).
      In bf16 mode blocks 2-4 read the bf16 twin of their input, as the engine's
      GEMM does.

    ``x``: the (B,3,N) device input as the model received it (any strides);
    ``init``: the state_dict before the step (BN running statistics of eval
    blocks). Returns {block: (gap, flip)}."""
    import torch
    import oracle
    from oracle import reference as R
    if tol is None:
        tol = 2e-3 if bf16 else 1e-5
    xcat = cap["xcat"]
    x16 = cap.get("xcat16")
    B, _, N = x.shape
    M, total = xcat.shape
    widths = [int(init[f"conv{i}.0.weight"].shape[0]) for i in range(1, 5)]
    dev = xcat.device
    xcat_cpu = xcat.detach().cpu()   # point-major rows: the oracle reads C-contiguous columns fast
    out = {}
    off_in = None
    for l in range(4):
        idx, arg, zpos = cap[("fwd", l)]
        if l == 0:
            xin = x.detach().float()
            want = oracle.knn(xin.cpu(), k)
            xin64 = xin.double()
        else:
            cin = widths[l - 1]
            view = xcat_cpu[:, off_in:off_in + cin].view(B, N, cin).permute(0, 2, 1)   # (B, C, N) view
            want = oracle.knn(view, k, order=oracle.ORDER_STRIDED)
            src = x16 if (bf16 and x16 is not None and x16.numel()) else xcat
            xin64 = src.detach()[:, off_in:off_in + cin].double().view(B, N, cin).permute(0, 2, 1)
        got = idx.view(B, N, k).long().cpu().numpy()
        np.testing.assert_array_equal(got, want, err_msg=f"block {l + 1} kNN differs from the oracle")
        i = l + 1
        w = init[f"conv{i}.0.weight"].to(dev).double()
        bn = {n: init[f"conv{i}.1.{n}"].to(dev).double() for n in ("weight", "bias", "running_mean", "running_var")}
        with torch.no_grad():
            e = R.graph_feature(xin64, k, idx=idx.to(dev).long().view(B, N, k))
            y = torch.nn.functional.conv2d(e, w)
            del e
            z = torch.nn.functional.batch_norm(y, bn["running_mean"].clone(), bn["running_var"].clone(), bn["weight"],
                                               bn["bias"], training[l], 0.1, 1e-5)
            del y
            out[i] = check_decisions(z, arg, zpos, B, N, tol)
            del z
        off_in = sum(widths[:l])
    return out


def edge_mlp_decisions(cap, B, N, k, w2, slope1=0.2, tol=1e-5):
    """Routing decisions of one engine edge_mlp2 forward (debug capture
    ``cap["emlp"]``, dgx.edgemlp._capture) for oracle.reference.edge_mlp2_routed,
    after validating them (reference models/layers.py:45-52):

    * conv2's max slot: recompute every edge's pre-BN conv2 value from the
      engine's own PQ / BN1 affine with the engine's arithmetic (h1 formula of
      the kernel that ran, bf16 operands in the fused bf16 kernel) in fp64 and
      require the chosen slot to be a maximum of sign(gamma2)·y2 over k up to
      ``tol`` of the scale; the captured selected value must be that slot's;
    * conv2's LeakyReLU sign: may only disagree with the recomputed BN2 output
      where it is below ``tol`` of the scale.

    Returns (zpos1 (B,C1,N,k), arg2 (B*N,C2), zpos2 (B*N,C2), (gap, flip));
    zpos1 = sign of BN1's output as the backward evaluates it (fma(a1, P_j + Q_i,
    b1)), the decision that routes conv1's gradient."""
    import torch
    c = cap["emlp"]
    PQ = c["PQ"].double()
    dev = PQ.device
    M = B * N
    C1 = PQ.shape[1] // 2
    C2 = c["arg"].shape[1]
    gid = c["idx"].long().view(M, k) + (torch.arange(M, device=dev) // N * N).view(M, 1)
    P = PQ[gid.reshape(-1), :C1].view(M, k, C1)
    Q = PQ[:, C1:].reshape(M, 1, C1)
    a1, b1 = c["a1"].double(), c["b1"].double()
    y1 = (P + Q).float().double()                       # the fp32 sum P_j + Q_i
    zpos1 = (a1 * y1 + b1 > 0).view(B, N, k, C1).permute(0, 3, 1, 2)
    if c["fused"]:   # emlp_fwd_kernel: fma(a1, P_j, fma(a1, Q_i, b1)), bf16 into the MFMA
        z1 = (a1 * P + (a1 * Q + b1).float().double()).float()
    else:            # mlp_h1_kernel: fma(a1, P_j + Q_i, b1)
        z1 = (a1 * y1 + b1).float()
    del P, y1
    h1 = torch.where(z1 > 0, z1, z1 * slope1)
    del z1
    W = w2.detach().reshape(C2, C1).float()
    if c["fused"]:
        h1, W = h1.bfloat16(), W.bfloat16()
    y2 = torch.matmul(h1.double(), W.double().t())      # (M, k, C2)
    del h1
    a2, b2 = c["a2"].double(), c["b2"].double()
    sgn = torch.where(a2 < 0, -1.0, 1.0).double()
    v = y2 * sgn
    scale = float(y2.abs().max())
    arg = c["arg"].long()
    vsel = torch.gather(v, 1, arg.unsqueeze(1)).squeeze(1)
    gap = float((v.max(dim=1)[0] - vsel).max()) / scale
    assert gap <= tol, ("conv2 max slot", gap, tol)
    ysel_c = vsel * sgn
    assert float((ysel_c - c["ysel"].double()).abs().max()) <= tol * scale, "captured selected value"
    zpos2 = (a2 * c["ysel"].double() + b2) > 0
    z2 = a2 * ysel_c + b2
    bad = zpos2 != (z2 > 0)
    zscale = float(z2.abs().max())
    flip = float(z2[bad].abs().max()) / zscale if bad.any() else 0.0
    assert flip <= tol, ("conv2 LeakyReLU sign", flip, tol)
    return zpos1, c["arg"], zpos2, (gap, flip)


def assert_knn_equivalent(idx, vals, ref_idx, ref_vals):
    """kNN parity with the reference: selected distance values bit-exact, and
    indices identical except inside the tie group at the k-th value, where the
    reference's torch.topk picks arbitrary members and dgx picks the smallest
    indices (canonical). Inside that group our indices must be ascending."""
    idx, ref_idx = np.asarray(idx), np.asarray(ref_idx)
    vals, ref_vals = np.asarray(vals), np.asarray(ref_vals)
    np.testing.assert_array_equal(vals, ref_vals)
    kth = ref_vals[..., -1:]
    strict = ref_vals > kth
    np.testing.assert_array_equal(np.where(strict, idx, -1), np.where(strict, ref_idx, -1))
    # every run of equal values (anywhere in the row) must list indices ascending
    eq = vals[..., 1:] == vals[..., :-1]
    assert (np.diff(idx, axis=-1)[eq] > 0).all()
