"""The CPU oracle is pinned against vectors produced by the reference itself
(tests/golden/make_goldens.py). CPU-only."""
import hashlib
import json
import os
import types

import numpy as np
import pytest
import torch

import oracle
from oracle import reference as R
from conftest import GOLDEN, rel_err, assert_knn_equivalent
from dgx import synth

KNN_CASES = ["c3", "c9", "c64", "c128", "c3k40", "c64k32", "c3n1000"]


def _x_view(pts, layout):
    t = torch.from_numpy(pts)
    return t.permute(0, 2, 1) if layout == "perm" else t.permute(0, 2, 1).contiguous()


@pytest.mark.parametrize("layout", ["bcn", "perm"])
@pytest.mark.parametrize("case", KNN_CASES)
def test_oracle_knn_matches_reference(golden, case, layout):
    g = golden("knn_cases.npz")
    key = f"{case}_{layout}"
    x = _x_view(g[key + "_x"], layout)
    k = g[key + "_idx"].shape[-1]
    idx, vals = oracle.knn(x, k, return_values=True)
    np.testing.assert_array_equal(idx, g[key + "_idx"])
    np.testing.assert_array_equal(vals, g[key + "_val"])  # bit-exact distances


def test_oracle_knn_ties(golden):
    g = golden("knn_cases.npz")
    x = _x_view(g["ties_perm_x"], "perm")
    idx, vals = oracle.knn(x, 20, return_values=True)
    assert_knn_equivalent(idx, vals, g["ties_perm_idx"], g["ties_perm_val"])
    assert (idx != g["ties_perm_idx"]).any()  # the fixture really has boundary ties


def test_oracle_sqnorm_orders_differ():
    # the layout-dependent rounding order is real: both orders are needed
    pts = synth.relu_normal(5, (1, 512, 64))
    a = oracle.sqnorm(_x_view(pts, "bcn"))
    b = oracle.sqnorm(_x_view(pts, "perm"))
    assert (a != b).any()


@pytest.mark.parametrize("name", ["xyz", "feat"])
def test_oracle_graph_feature(golden, name):
    g = golden("graph_feature.npz")
    x, idx = g[name + "_x"], g[name + "_idx"]
    np.testing.assert_array_equal(oracle.graph_feature(x, idx), g[name + "_cat"])
    np.testing.assert_array_equal(oracle.graph_feature(x, idx, disp_only=True), g[name + "_disp"])
    np.testing.assert_array_equal(oracle.graph_feature(x, idx, knn_only=True), g[name + "_knn"])
    t = torch.from_numpy(x)
    np.testing.assert_array_equal(R.graph_feature(t, idx=torch.from_numpy(idx).long()).numpy(), g[name + "_cat"])


def test_reference_restatement_edgeconv_block(golden):
    g = golden("edgeconv_block.npz")
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    w = torch.from_numpy(g["weight"]).requires_grad_(True)
    gamma = torch.from_numpy(g["gamma"]).requires_grad_(True)
    beta = torch.from_numpy(g["beta"]).requires_grad_(True)
    co = w.shape[0]
    bn = {"weight": gamma, "bias": beta, "running_mean": torch.zeros(co), "running_var": torch.ones(co)}
    k = int(g["k"])
    y = R.edgeconv_block(x, k, w, bn, True, idx=torch.from_numpy(g["idx"]).long())
    y.backward(torch.from_numpy(g["gout"]))
    assert rel_err(y.detach(), g["out"]) < 1e-6
    assert rel_err(x.grad, g["dx"]) < 1e-5
    assert rel_err(w.grad, g["dweight"]) < 1e-5
    assert rel_err(gamma.grad, g["dgamma"]) < 1e-5
    assert rel_err(beta.grad, g["dbeta"]) < 1e-5
    assert rel_err(bn["running_mean"], g["running_mean"]) < 1e-6
    assert rel_err(bn["running_var"], g["running_var"]) < 1e-6


def test_reference_restatement_dgcnn(golden):
    g = golden("dgcnn_small.npz")
    params = {k[5:]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith("init.")}
    for n, t in params.items():
        if t.dtype == torch.float32 and "running" not in n:
            t.requires_grad_(True)
    y, _ = R.dgcnn(torch.from_numpy(g["x"]), 10, params, training=True)
    y.backward(torch.from_numpy(g["gout"]))
    assert rel_err(y.detach(), g["out"]) < 1e-5
    for k in g.files:
        if k.startswith("grad."):
            assert rel_err(params[k[5:]].grad, g[k]) < 1e-4, k
        if k.startswith("after."):
            assert rel_err(params[k[6:]], g[k]) < 1e-5, k


def test_full_size_knn_hashes():
    """The oracle reproduces the reference's canonical kNN of the bench inputs."""
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        H = json.load(f)
    gens = {"cfg2_layer1": lambda: synth.cube_clouds(32, 1024, 0),
            "ties_layer1": lambda: synth.tie_clouds(32, 1024, 1)}
    for name, gen in gens.items():
        h = H[name]
        pts = gen()
        assert hashlib.sha256(pts.tobytes()).hexdigest() == h["input_sha256"]
        idx, vals = oracle.knn(torch.from_numpy(pts).permute(0, 2, 1), h["k"], return_values=True)
        assert hashlib.sha256(vals.tobytes()).hexdigest() == h["val_sha256"], name
        if name != "ties_layer1":
            assert hashlib.sha256(idx.astype(np.int32).tobytes()).hexdigest() == h["idx_sha256"], name


def test_synth_generator_pinned():
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        H = json.load(f)
    assert hashlib.sha256(synth.cube_clouds(32, 2048, 0).tobytes()).hexdigest() == H["cfg3_layer1"]["input_sha256"]
    assert hashlib.sha256(synth.s3dis_blocks(24, 4096, 2).tobytes()).hexdigest() == H["cfg5_layer1"]["input_sha256"]
