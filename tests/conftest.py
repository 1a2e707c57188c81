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
