"""Push form of the EdgeConv backward scatter (dgx_edge_bwd_scatter_push_f32;
the autograd of dgcnn.py:84-98's gather + max through BN, the reverse of
get_graph_feature's index at dgcnn.py:33-36). Each source's selected dz is
added to its target in 64-bit fixed point, so:

* against an fp64 restatement of the same scatter (every term summed in fp64)
  the push result is within fp32 rounding (2e-6 of the output scale), and so
  is the pull form it replaces;
* it is deterministic (two launches bitwise equal) including at hubs, where
  hundreds of sources select one target;
* all modes of the entry (finalize in the prologue or c0 / c1 given, packed
  dz|slot words or dz + slot bytes, fp32 or bf16 output) and the slice
  geometries (channels not a multiple of 8, N needing several point parts or
  narrow slices) agree with the pull form;
* a channel with a non-finite dz turns into NaN (the fp16 GradScaler's
  overflow check still sees it), the other channels are untouched."""

import pytest
import torch

from dgx import _native as nat
from dgx import bn as bn_
from dgx import edgeconv as E

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


def _setup(cuda, B, N, k, Co, hubs=False, seed=0, packed=False):
    g = torch.Generator(device="cpu").manual_seed(seed + N + Co)
    M = B * N
    L = nat.lib()
    PQ = torch.randn(M, 2 * Co, generator=g).to(cuda)
    if hubs:   # three in four neighbours are one of 4 hub points: in-degrees in the thousands
        idx = torch.where(torch.rand(B, N, k, generator=g) < 0.75, torch.randint(0, 4, (B, N, k), generator=g),
                          torch.randint(0, N, (B, N, k), generator=g)).to(torch.int32).to(cuda)
    else:
        idx = torch.randint(0, N, (B, N, k), generator=g, dtype=torch.int32).to(cuda)
    gamma = torch.randn(Co, generator=g).to(cuda)
    stream = nat.stream_of(PQ)
    ysel, arg, sumP, part, prow = E.edge_select(PQ, idx, B, N, k, Co, gamma, stream)
    bn = torch.nn.BatchNorm2d(Co).to(cuda).train()
    st = bn_.batch_stats(part, prow, float(M * k), bn, gamma, torch.zeros_like(gamma), stream)
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
    c = bn_.backward_consts(partials, nblk, float(M * k), st, stream)
    return dict(L=L, B=B, N=N, k=k, Co=Co, M=M, PQ=PQ, idx=idx, arg=arg, sumP=sumP, st=st, dz=dz, partials=partials,
                nblk=nblk, rowptr=rowptr, edges=edges, c0=c[2], c1=c[3], stream=stream)


def _push(S, packed, bf16=False, fin=False, dz=None):
    L, st = S["L"], S["st"]
    out = torch.empty(S["M"], 2 * S["Co"], device=S["PQ"].device, dtype=torch.bfloat16 if bf16 else torch.float32)
    o = [torch.full((S["Co"],), float("nan"), device=out.device) for _ in range(4)]
    c0, c1 = (o[2], o[3]) if fin else (S["c0"], S["c1"])
    nat.check(L.dgx_edge_bwd_scatter_push_f32(
        nat.f32(S["PQ"]), 2 * S["Co"], nat.i32(S["idx"]), nat.i32(S["rowptr"]), nat.i32(S["edges"]),
        nat.f32(S["dz"] if dz is None else dz), None if packed else nat.u8(S["arg"]), nat.f32(S["sumP"]), S["B"],
        S["N"], S["k"], S["Co"], nat.f32(S["partials"]) if fin else None, S["nblk"] if fin else 0,
        float(S["M"] * S["k"]), nat.f32(st.scale), nat.f32(st.mean), nat.f32(st.invstd), 0,
        *((nat.f32(o[0]), nat.f32(o[1])) if fin else (None, None)), nat.f32(c0), nat.f32(c1),
        nat.ptr(out, nat.F32, nat.BF16), int(bf16), int(packed), S["stream"]), "scatter push")
    return out, o


def _pull(S, packed):
    L, st = S["L"], S["st"]
    out = torch.empty(S["M"], 2 * S["Co"], device=S["PQ"].device)
    common = (S["B"], S["N"], S["k"], S["Co"], nat.f32(st.scale), nat.f32(S["c0"]), nat.f32(S["c1"]), nat.f32(out), 0,
              S["stream"])
    if packed:
        nat.check(L.dgx_edge_bwd_scatter_packed_f32(nat.f32(S["PQ"]), 2 * S["Co"], nat.i32(S["rowptr"]),
                                                    nat.i32(S["edges"]), nat.f32(S["dz"]), nat.f32(S["sumP"]),
                                                    *common), "scatter")
    else:
        nat.check(L.dgx_edge_bwd_scatter_f32(nat.f32(S["PQ"]), 2 * S["Co"], nat.i32(S["rowptr"]), nat.i32(S["edges"]),
                                             nat.f32(S["dz"]), nat.u8(S["arg"]), nat.f32(S["sumP"]), *common),
                  "scatter")
    return out


def _ref64(S, packed):
    """dP_j = a sum_{(i,s): idx[i][s] = j, arg[i][c] = s} dz_i[c] + sum_{idx[i][s] = j} (c0 + c1 (P_j + Q_i)),
    dQ_i = a dz_i + k c0 + c1 (k Q_i + sum_s P_idx[i][s]), every term in fp64."""
    B, N, k, Co, M = S["B"], S["N"], S["k"], S["Co"], S["M"]
    PQ = S["PQ"].double()
    P, Q = PQ[:, :Co], PQ[:, Co:]
    dz = S["dz"]
    if packed:
        dz = (dz.view(torch.int32) & ~63).view(torch.float32)
    dz = dz.double()
    a, c0, c1 = S["st"].scale.double(), S["c0"].double(), S["c1"].double()
    gidx = (S["idx"].long() + (torch.arange(B, device=PQ.device) * N).view(B, 1, 1)).view(M, k)
    jsel = torch.gather(gidx, 1, S["arg"].long())                     # (M, Co): the selected target per channel
    sd = torch.zeros(M, Co, dtype=torch.float64, device=PQ.device).scatter_add_(0, jsel, dz)
    deg = torch.bincount(gidx.flatten(), minlength=M).double().unsqueeze(1)
    sq = torch.zeros(M, Co, dtype=torch.float64, device=PQ.device).index_add_(0, gidx.flatten(),
                                                                               Q.repeat_interleave(k, 0))
    dP = a * sd + c0 * deg + c1 * (deg * P + sq)
    dQ = a * dz + k * c0 + c1 * (k * Q + P[gidx].sum(1))
    return torch.cat([dP, dQ], 1)


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("B,N,k,Co,hubs", [(32, 1024, 20, 64, False), (4, 777, 11, 20, False),
                                           (8, 1024, 20, 256, True), (2, 2048, 40, 64, False),
                                           (1, 12000, 16, 8, False)])
def test_push_matches_fp64_and_pull(cuda, B, N, k, Co, hubs, packed):
    S = _setup(cuda, B, N, k, Co, hubs=hubs, packed=packed)
    ref = _ref64(S, packed)
    push, _ = _push(S, packed)
    push2, _ = _push(S, packed)
    pull = _pull(S, packed)
    torch.cuda.synchronize()
    e_push, e_pull = _rel(push, ref), _rel(pull, ref)
    print(f"B{B} N{N} k{k} Co{Co} hubs={hubs} packed={packed}: push {e_push:.2e} pull {e_pull:.2e}")
    assert torch.equal(push, push2)                  # order-independent sums: bitwise repeatable
    assert e_push < 2e-6 and e_pull < 2e-6
    assert _rel(push, pull) < 4e-6


@pytest.mark.parametrize("packed", [False, True])
def test_push_finalize_and_bf16_output(cuda, packed):
    """partials given: the prologue finalize writes dgamma / dbeta / c0 / c1 as
    the separate finalize does (1e-6, fp64 order), dPQ as with given c0 / c1;
    bf16 output = the fp32 result rounded."""
    S = _setup(cuda, 16, 1024, 20, 128, packed=packed, seed=3)
    out_fin, o = _push(S, packed, fin=True)
    out, _ = _push(S, packed)
    out16, _ = _push(S, packed, bf16=True)
    torch.cuda.synchronize()
    dgamma, dbeta, c0, c1 = bn_.backward_consts(S["partials"], S["nblk"], float(S["M"] * S["k"]), S["st"],
                                                S["stream"])
    for a, b in zip((dgamma, dbeta, c0, c1), o):
        assert _rel(b, a) < 1e-6
    assert _rel(out_fin, out) < 1e-5
    if torch.equal(o[2], c0) and torch.equal(o[3], c1):
        assert torch.equal(out_fin, out)
    assert torch.equal(out16, out.to(torch.bfloat16))


def test_push_nonfinite_channel(cuda):
    S = _setup(cuda, 4, 512, 20, 16, seed=7)
    dz = S["dz"].clone()
    dz[37, 5] = float("inf")
    out, _ = _push(S, False, dz=dz)
    ref, _ = _push(S, False)
    torch.cuda.synchronize()
    Co = S["Co"]
    b = 37 // S["N"]
    rows = slice(b * S["N"], (b + 1) * S["N"])
    assert torch.isnan(out[rows, 5]).all()                       # dP of the channel, the cloud of the inf
    keep = torch.ones(2 * Co, dtype=torch.bool)
    keep[5] = False
    keep[Co + 5] = False
    assert torch.equal(out[:, keep], ref[:, keep])


@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("B,N,k,Co", [(8, 1024, 20, 64), (4, 777, 11, 20)])
def test_pull_split_planes_output(cuda, packed, B, N, k, Co, mode):
    """out_bf16 = 2 / 3 (the fp32 mode's split class): the pull scatter writes dPQ
    as its (hi, lo) bf16 planes, lo at + B*N*2Co (mode 3: hi again at + 2 B*N*2Co)
    — bitwise the fp32 output split by dgx_split_bf16's rounding (hi = bf16(v),
    lo = bf16(v - hi)); the push form refuses both."""
    S = _setup(cuda, B, N, k, Co, packed=packed, seed=5)
    L, st = S["L"], S["st"]
    ref = _pull(S, packed)
    planes = torch.zeros(3, S["M"], 2 * Co, device=cuda, dtype=torch.bfloat16)
    common = (B, N, k, Co, nat.f32(st.scale), nat.f32(S["c0"]), nat.f32(S["c1"]), nat.ptr(planes, nat.BF16), mode,
              S["stream"])
    if packed:
        nat.check(L.dgx_edge_bwd_scatter_packed_f32(nat.f32(S["PQ"]), 2 * Co, nat.i32(S["rowptr"]), nat.i32(S["edges"]),
                                                    nat.f32(S["dz"]), nat.f32(S["sumP"]), *common), "scatter split")
    else:
        nat.check(L.dgx_edge_bwd_scatter_f32(nat.f32(S["PQ"]), 2 * Co, nat.i32(S["rowptr"]), nat.i32(S["edges"]),
                                             nat.f32(S["dz"]), nat.u8(S["arg"]), nat.f32(S["sumP"]), *common),
                  "scatter split")
    torch.cuda.synchronize()
    hi = ref.to(torch.bfloat16)
    lo = (ref - hi.float()).to(torch.bfloat16)
    assert torch.equal(planes[0], hi) and torch.equal(planes[1], lo)
    assert torch.equal(planes[2], hi if mode == 3 else torch.zeros_like(hi))
    with pytest.raises(RuntimeError):
        _push(S, packed, bf16=mode)
