"""a2 parity: get_graph_feature (HIP gather) vs the reference's goldens."""
import numpy as np
import pytest
import torch

from conftest import rel_err
from oracle import reference as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["xyz", "feat"])
def test_graph_feature_golden(golden, cuda, name):
    from models.dgcnn import get_graph_feature
    g = golden("graph_feature.npz")
    x = torch.from_numpy(g[name + "_x"]).to(cuda)
    np.testing.assert_array_equal(get_graph_feature(x, k=8).cpu().numpy(), g[name + "_cat"])
    np.testing.assert_array_equal(get_graph_feature(x, k=8, disp_only=True).cpu().numpy(), g[name + "_disp"])
    np.testing.assert_array_equal(get_graph_feature(x, k=8, knn_only=True).cpu().numpy(), g[name + "_knn"])


@pytest.mark.parametrize("mode", ["cat", "disp", "knn"])
def test_graph_feature_backward(cuda, mode):
    from models.dgcnn import get_graph_feature, knn
    torch.manual_seed(0)
    x = torch.randn(2, 5, 70)
    kw = {"knn_only": mode == "knn", "disp_only": mode == "disp"}
    xg = x.to(cuda).requires_grad_(True)
    out = get_graph_feature(xg, k=6, **kw)
    gout = torch.randn(out.shape)
    out.backward(gout.to(cuda))
    idx = knn(x.to(cuda), 6).cpu()
    xc = x.clone().requires_grad_(True)
    ref = R.graph_feature(xc, 6, idx=idx, **kw)
    ref.backward(gout)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), ref.detach().numpy())
    assert rel_err(xg.grad.cpu(), xc.grad) < 1e-6
