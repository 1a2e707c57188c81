"""Reverse kNN graph (dgx_graph_reverse): the CSR of in-edges the EdgeConv
backward scatters through (the index_put_(accumulate) of reference
models/dgcnn.py:33 under autograd). Checked exactly against numpy: every list
ascending by edge id ((global source << 6) | slot), on random graphs, on
degenerate ones (every point has the same neighbours: one range overflows the
workgroup's LDS capacity) and at the bench size."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _reference(idx):
    B, N, k = idx.shape
    src = np.repeat(np.arange(B * N, dtype=np.int64), k)
    slot = np.tile(np.arange(k, dtype=np.int64), B * N)
    tgt = (idx.reshape(B, N * k) + (np.arange(B)[:, None] * N)).reshape(-1).astype(np.int64)
    ids = (src << 6) | slot
    order = np.lexsort((ids, tgt))
    edges = ids[order].astype(np.int32)
    rowptr = np.concatenate([[0], np.cumsum(np.bincount(tgt, minlength=B * N))]).astype(np.int32)
    return rowptr, edges


def _run(idx, cuda):
    from dgx import _native as nat
    B, N, k = idx.shape
    t = torch.from_numpy(idx).to(cuda)
    rowptr = torch.full((B * N + 1,), -7, dtype=torch.int32, device=cuda)
    edges = torch.full((B * N * k,), -7, dtype=torch.int32, device=cuda)
    with torch.cuda.device(cuda):
        nat.check(nat.lib().dgx_graph_reverse(nat.ptr(t), B, N, k, nat.ptr(rowptr), nat.ptr(edges),
                                              nat.stream_of(t)), "reverse")
    return rowptr.cpu().numpy(), edges.cpu().numpy()


def _random_graph(B, N, k, seed):
    rng = np.random.default_rng(seed)
    return np.stack([np.stack([rng.choice(N, k, replace=False) for _ in range(N)]) for _ in range(B)]).astype(np.int32)


@pytest.mark.parametrize("B,N,k", [(2, 100, 7), (3, 1024, 20), (1, 2048, 40), (2, 33, 33), (1, 5, 1)])
def test_reverse_graph_random(cuda, B, N, k):
    idx = _random_graph(B, N, k, B * 1000 + N + k)
    rp, ed = _run(idx, cuda)
    ref_rp, ref_ed = _reference(idx)
    np.testing.assert_array_equal(rp, ref_rp)
    np.testing.assert_array_equal(ed, ref_ed)


@pytest.mark.parametrize("N,k", [(1024, 20), (4096, 20), (2048, 40)])
def test_reverse_graph_degenerate(cuda, N, k):
    """All points equal: every point's kNN is 0..k-1 (canonical ties), so k
    targets receive N in-edges each."""
    idx = np.tile(np.arange(k, dtype=np.int32), (2, N, 1))
    rp, ed = _run(idx, cuda)
    ref_rp, ref_ed = _reference(idx)
    np.testing.assert_array_equal(rp, ref_rp)
    np.testing.assert_array_equal(ed, ref_ed)


def test_reverse_graph_bench_size_from_knn(cuda):
    from dgx import synth
    from models.dgcnn import knn
    x = torch.from_numpy(synth.cube_clouds(32, 1024, 0)).to(cuda).permute(0, 2, 1)
    idx = knn(x, 20).to(torch.int32).cpu().numpy()
    rp, ed = _run(idx, cuda)
    ref_rp, ref_ed = _reference(idx)
    np.testing.assert_array_equal(rp, ref_rp)
    np.testing.assert_array_equal(ed, ref_ed)
