"""In-launch BatchNorm finalize of the EdgeConv block's backward (dgcnn.py:54-73,
the BN of each block's Conv2d): the backward scatter's prologue finalize
(dgx_edge_bwd_scatter_fin_f32) against the separate-launch path on the same
inputs. The statistics differ only by the fp64 summation order of the same
fp32 partials, so they are held to 1e-6 relative; dPQ must match exactly."""


import pytest
import torch

from dgx import _native as nat
from dgx import bn as bn_
from dgx import edgeconv as E

pytestmark = pytest.mark.gpu

TOL = 1e-6


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("B,N,k,Co,ev", [(32, 1024, 20, 64, False), (4, 777, 11, 24, False), (8, 1024, 20, 128, True)])
def test_backward_scatter_finalize(cuda, B, N, k, Co, ev, packed):
    g = torch.Generator(device="cpu").manual_seed(N + Co)
    M = B * N
    L = nat.lib()
    PQ = torch.randn(M, 2 * Co, generator=g).to(cuda)
    idx = torch.randint(0, N, (B, N, k), generator=g, dtype=torch.int32).to(cuda)
    gamma = torch.randn(Co, generator=g).to(cuda)
    stream = nat.stream_of(PQ)
    ysel, arg, sumP, part, prow = E.edge_select(PQ, idx, B, N, k, Co, gamma, stream)
    bn = torch.nn.BatchNorm2d(Co).to(cuda).train()
    st = bn_.batch_stats(part, prow, float(M * k), bn, gamma, torch.zeros_like(gamma), stream)
    if ev:
        st = st._replace(eval=True)
    dY = torch.randn(M, Co, generator=g).to(cuda)
    nblk = max(1, min(1024, (M + 63) // 64))
    dz = torch.empty(M, Co, device=cuda)
    partials = torch.empty(nblk, 2, Co, device=cuda)
    bn_args = (M, Co, nat.f32(st.scale), nat.f32(st.shift), nat.f32(st.mean), nat.f32(st.invstd), 0.2, nat.f32(dz),
               nat.f32(partials), nblk, stream)
    if packed:
        nat.check(L.dgx_edge_bwd_dz_packed_f32(nat.f32(dY), Co, nat.f32(ysel), nat.u8(arg), *bn_args), "dz")
    else:
        nat.check(L.dgx_edge_bwd_dz_f32(nat.f32(dY), Co, nat.f32(ysel), *bn_args), "dz")
    (rowptr, edges), = E._reverse_graphs([idx], B, N, k, cuda)
    dgamma, dbeta, c0, c1 = bn_.backward_consts(partials, nblk, float(M * k), st, stream)
    ref = torch.empty(M, 2 * Co, device=cuda)
    common = (B, N, k, Co, nat.f32(st.scale), nat.f32(c0), nat.f32(c1), nat.f32(ref), 0, stream)
    if packed:
        nat.check(L.dgx_edge_bwd_scatter_packed_f32(nat.f32(PQ), 2 * Co, nat.i32(rowptr), nat.i32(edges),
                                                    nat.f32(dz), nat.f32(sumP), *common), "scatter")
    else:
        nat.check(L.dgx_edge_bwd_scatter_f32(nat.f32(PQ), 2 * Co, nat.i32(rowptr), nat.i32(edges), nat.f32(dz),
                                             nat.u8(arg), nat.f32(sumP), *common), "scatter")
    out = torch.empty(M, 2 * Co, device=cuda)
    o = [torch.full((Co,), float("nan"), device=cuda) for _ in range(4)]
    nat.check(L.dgx_edge_bwd_scatter_fin_f32(
        nat.f32(PQ), 2 * Co, nat.i32(rowptr), nat.i32(edges), nat.f32(dz), None if packed else nat.u8(arg),
        nat.f32(sumP), B, N, k, Co, nat.f32(partials), nblk, float(M * k), nat.f32(st.scale), nat.f32(st.mean),
        nat.f32(st.invstd), int(ev), *(nat.f32(t) for t in o), nat.f32(out), 0, int(packed), stream), "scatter fin")
    torch.cuda.synchronize()
    for a, b in zip((dgamma, dbeta, c0, c1), o):
        assert _rel(b, a) < TOL
    if ev:
        assert float(o[2].abs().max()) == 0.0 and float(o[3].abs().max()) == 0.0
    # dPQ from (nearly) the same c0 / c1: equal up to their last-bit differences
    assert _rel(out, ref) < 1e-5
    if torch.equal(o[2], c0) and torch.equal(o[3], c1):
        assert torch.equal(out, ref)


def test_packed_dz_words(cuda):
    """dgx_edge_bwd_dz_packed_f32: each word = dz with its 6 low mantissa bits
    replaced by the selected slot; the partials are those of the exact dz."""
    B, N, Co, k = 4, 300, 48, 20
    M = B * N
    L = nat.lib()
    g = torch.Generator(device="cpu").manual_seed(5)
    ysel = torch.randn(M, Co, generator=g).to(cuda)
    arg = torch.randint(0, k, (M, Co), generator=g, dtype=torch.uint8).to(cuda)
    dY = torch.randn(M, Co, generator=g).to(cuda)
    sc, sh, mu, ist = (torch.randn(Co, generator=g).to(cuda) for _ in range(4))
    outs = []
    for packed in (False, True):
        dz = torch.empty(M, Co, device=cuda)
        part = torch.empty(16, 2, Co, device=cuda)
        a = (M, Co, nat.f32(sc), nat.f32(sh), nat.f32(mu), nat.f32(ist), 0.2, nat.f32(dz), nat.f32(part), 16,
             nat.stream_of(dz))
        if packed:
            nat.check(L.dgx_edge_bwd_dz_packed_f32(nat.f32(dY), Co, nat.f32(ysel), nat.u8(arg), *a), "dz packed")
        else:
            nat.check(L.dgx_edge_bwd_dz_f32(nat.f32(dY), Co, nat.f32(ysel), *a), "dz")
        outs.append((dz, part))
    (dz, p0), (dzp, p1) = outs
    w = dzp.view(torch.int32)
    assert torch.equal(w & 63, arg.to(torch.int32))
    assert torch.equal(w & ~63, dz.view(torch.int32) & ~63)
    assert torch.equal(p0, p1)
