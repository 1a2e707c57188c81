"""CPU checks of the boundary: libdgx.so loads and exports every symbol that
include/dgx.h declares; the Python mirror binds them; no silent CPU path."""
import ctypes
import os
import re
import types

import pytest
import torch

from conftest import REPO


def _declared():
    with open(os.path.join(REPO, "include", "dgx.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(dgx_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    from dgx import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    declared = _declared()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    # the Python binding declares a signature for every exported symbol
    assert sorted(_native.exported_symbols()) == declared


def test_version_and_errors():
    from dgx import _native
    L = _native.lib()
    assert L.dgx_version().decode().startswith("dgx")
    assert L.dgx_strerror(-1).decode() == "invalid argument"
    # argument validation happens before any device work
    assert L.dgx_knn_f32(None, 0, 0, 0, 1, 3, 8, 2, 0, None, None, None, 0, None) == -1
    # |x|^2 (B*N floats) + operand image per cloud: 32-point tiles x 64 lanes x NS = ceil(C/2) (rounded
    # to 2, 4, 8, ...) MFMA steps + 32 norms per tile (C=64: 32 tiles x 64 x 32 + 32 x 32)
    assert L.dgx_knn_workspace_bytes(2, 64, 1024) == 2 * 1024 * 4 + 2 * (32 * 64 * 32 + 32 * 32) * 4
    # |x|^2 (B*N floats) + operand image (64 tiles x 64 lanes x 16 floats + 64 x 16 norms per cloud at C=64)
    assert L.dgx_knn_workspace_bytes(2, 64, 1024) == 2 * 1024 * 4 + 2 * (64 * 64 * 16 + 64 * 16) * 4
    assert L.dgx_knn_image_bytes(2, 3, 1000) == 2 * (63 * 64 * 1 + 63 * 16) * 4


def test_host_tensors_take_the_cpu_path_without_libdgx(monkeypatch):
    """Host tensors are served by dgx.cpu and never reach the
    HIP library: with libdgx.so made unloadable the drop-in still runs on the
    CPU, while the device-only entry points keep rejecting host tensors."""
    from dgx import _native as nat
    from models.dgcnn import DGCNN, knn, get_graph_feature

    def no_lib():
        raise ImportError("libdgx.so unavailable (test)")
    monkeypatch.setattr(nat, "lib", no_lib)
    x = torch.rand(2, 3, 32)
    assert knn(x, 4).shape == (2, 32, 4)
    assert get_graph_feature(x, k=4).shape == (2, 6, 32, 4)
    assert DGCNN(types.SimpleNamespace(emb_dim=64, k=4))(x).shape == (2, 64, 32)
    with pytest.raises(RuntimeError, match="ROCm device"):
        nat.require_device(x)


def test_state_dict_keys_match_reference():
    import json
    from conftest import GOLDEN
    from models.dgcnn import DGCNN
    from models.layers import PositionEmbedding
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        keys = json.load(f)["state_dict_keys"]
    assert list(DGCNN(types.SimpleNamespace(emb_dim=1024, k=20)).state_dict().keys()) == keys["DGCNN"]
    assert list(PositionEmbedding(types.SimpleNamespace(k=20)).state_dict().keys()) == keys["PositionEmbedding"]


def test_host_op_library_loads():
    """libdgx_torch.so (the C++ schedule + autograd layer over libdgx.so) loads
    and registers the torch.ops.dgx_host ops every device path runs; host
    tensors never take them."""
    from dgx import host
    from models.dgcnn import DGCNN
    host.load()
    want = {
        "dgcnn": "dgx_host::dgcnn(Tensor x, Tensor[] params, Tensor?[] bufs, float[] bn_f, int[] bn_i, str[] groups",
        "chain_forward": "dgx_host::chain_forward(Tensor x, int k, Tensor[] weights",
        "chain_backward": "dgx_host::chain_backward(Tensor dxcat, Tensor xcat, Tensor xcat16, Tensor[] saved",
        "pointconv_forward": "dgx_host::pointconv_forward(Tensor X, Tensor X16, int B, int N",
        "pointconv_backward": "dgx_host::pointconv_backward(Tensor dout, Tensor[] saved",
        "knn_timing": "dgx_host::knn_timing(bool on) -> float[]",
    }
    for name, head in want.items():
        assert str(getattr(torch.ops.dgx_host, name).default._schema).startswith(head), name
    assert torch.ops.dgx_host.knn_timing(False) == []
    assert not host.applies(DGCNN(types.SimpleNamespace(emb_dim=64, k=4)).train(), torch.rand(2, 3, 32))


def test_knn_shape_routing():
    """Shapes outside the fused kNN kernel route to the generic path (any C,
    k up to 8192, any N) instead of failing; its workspace query is exported."""
    from dgx import _native, ops
    assert ops.fast_shape(128, 64, 12288) and not ops.fast_shape(129, 20, 1024)
    assert not ops.fast_shape(3, 65, 1024) and not ops.fast_shape(3, 20, 12289)
    L = _native.lib()
    # |x|^2 (B*N, 16-byte rounded) + one chunk of dot rows (min(N, 2^24 / N rounded to 64) x N)
    assert L.dgx_knn_generic_workspace_bytes(2, 256, 1000) == (2000 + 1000 * 1000) * 4
