"""bf16 MFMA GEMMs (csrc/gemm.hip) against a plain fp32/fp64 PyTorch reference of
the same op on the bf16-rounded operands (the kernel rounds operands to bf16
RNE and accumulates in fp32, so only the summation order differs: 1e-5 rel).
Covers every layout/epilogue the engine launches, ragged M/N/K, the K=3 first
layer, column slices of the concat buffer, the fused BatchNorm statistics,
split-K slabs with the [W1;W2] -> [W1|W2] un-stacking, and determinism."""
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _bf(t):
    return t.to(torch.bfloat16).double()


def _ref(a, b):  # a (M,K), b (N,K) in fp64 of bf16-rounded values
    return (_bf(a) @ _bf(b).t()).cpu()


@pytest.mark.parametrize("M,N,K", [(32768, 1024, 512), (1000, 200, 64), (777, 128, 3), (130, 64, 45),
                                   (4096, 512, 128), (1, 1, 1)])
def test_xwt_store_and_stats(cuda, M, N, K):
    from dgx import gemm as G
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=cuda)
    w = torch.randn(N, K, device=cuda) * 0.1
    ref = _ref(x, w)
    z = G.mm_xwt(x, w)
    assert rel_err(z.cpu().numpy(), ref.numpy()) < TOL
    z2, part = G.mm_xwt(x, w, stats=True)
    assert torch.equal(z, z2)
    ps = part.double().sum(0).cpu()
    zd = z.double().cpu()
    assert rel_err(ps[0].numpy(), zd.sum(0).numpy()) < 1e-4
    assert rel_err(ps[1].numpy(), (zd * zd).sum(0).numpy()) < 1e-5


def test_xwt_strided_slice_of_concat_buffer(cuda):
    from dgx import gemm as G
    torch.manual_seed(1)
    xcat = torch.randn(3000, 512, device=cuda)
    X = xcat[:, 128:256]           # a block's input columns
    w = torch.randn(512, 128, device=cuda)
    assert rel_err(G.mm_xwt(X, w).cpu().numpy(), _ref(X, w).numpy()) < TOL
    xpm = torch.randn(2, 517, 3, device=cuda).reshape(-1, 3)  # first layer, K = 3, ld = 3
    w3 = torch.randn(128, 3, device=cuda)
    assert rel_err(G.mm_xwt(xpm, w3).cpu().numpy(), _ref(xpm, w3).numpy()) < TOL


@pytest.mark.parametrize("a_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(32768, 512, 1024), (1000, 64, 128), (333, 128, 512), (70, 3, 128)])
def test_xw_store_and_accumulate(cuda, a_dtype, M, N, K):
    from dgx import gemm as G
    torch.manual_seed(M * 7 + N)
    x = torch.randn(M, K, device=cuda).to(a_dtype)
    w = torch.randn(K, N, device=cuda) * 0.05
    ref = (_bf(x.float()) @ _bf(w)).cpu()
    y = G.mm_xw(x, w)
    assert rel_err(y.cpu().numpy(), ref.numpy()) < TOL
    base = torch.randn(M, N + 5, device=cuda)
    dst = base.clone()
    G.mm_xw(x, w, out=dst[:, 2:2 + N], accumulate=True)
    exp = base.double().cpu()
    exp[:, 2:2 + N] += ref
    assert rel_err(dst.cpu().numpy(), exp.numpy()) < TOL


@pytest.mark.parametrize("a_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("R,M,N", [(32768, 1024, 512), (32768, 512, 128), (5000, 128, 64), (999, 128, 3),
                                   (64, 40, 20), (32768, 128, 3), (2048, 600, 4), (77, 300, 1)])
def test_atb_split_k(cuda, a_dtype, R, M, N):
    from dgx import gemm as G
    torch.manual_seed(R + M)
    a = torch.randn(R, M, device=cuda).to(a_dtype)
    b = torch.randn(R, N, device=cuda)
    ref = (_bf(a.float()).t() @ _bf(b)).cpu()
    out = torch.empty(M, N, device=cuda)
    G.mm_atb(a, b, out)
    assert rel_err(out.cpu().numpy(), ref.numpy()) < TOL
    out2 = torch.empty(M, N, device=cuda)
    G.mm_atb(a, b, out2)
    assert torch.equal(out, out2), "split-K slab sum must be deterministic"


def test_atb_unstacks_edge_weight(cuda):
    """dW of an EdgeConv block: rows [0,Co) are the x_j half, rows [Co,2Co) the
    x_i half; the reference weight is (Co, 2C) = [W1 | W2] (dgcnn.py:55)."""
    from dgx import gemm as G
    torch.manual_seed(3)
    co, c, R = 64, 64, 4096
    dpq = torch.randn(R, 2 * co, device=cuda)
    X = torch.randn(R, 512, device=cuda)[:, 64:64 + c]
    full = (_bf(dpq).t() @ _bf(X)).cpu()
    gw = torch.empty(co, 2 * c, device=cuda)
    G.mm_atb(dpq, X, gw, split_rows=co)
    exp = torch.cat([full[:co], full[co:]], dim=1)
    assert rel_err(gw.cpu().numpy(), exp.numpy()) < TOL


def test_gemm_rejects_unsupported(cuda):
    from dgx import _native as nat
    x = torch.randn(16, 16, device=cuda)
    L = nat.lib()
    # (bf16 KC, fp32 KC) with accumulate is not a layout the engine launches
    rc = L.dgx_gemm_bf16(nat.ptr(x), 1, 0, 16, nat.ptr(x), 0, 0, 16, 16, 16, 16, 1, 1, nat.ptr(x), 16, None,
                         nat.stream_of(x))
    assert rc == -2
    assert L.dgx_gemm_bf16(None, 0, 0, 16, nat.ptr(x), 0, 0, 16, 16, 16, 16, 0, 1, nat.ptr(x), 16, None,
                           nat.stream_of(x)) == -1


# ---- bf16-operand path: LDS-DMA staging (global_load_lds), transposed reads ----

@pytest.mark.parametrize("M,N,K", [(32768, 1024, 512), (32768, 512, 1024), (65536 + 300, 256, 64), (1000, 128, 64),
                                   (777, 64, 128), (3000, 512, 1024), (129, 200, 192)])
def test_lds_xwt_store_stats_addend(cuda, M, N, K):
    from dgx import gemm as G
    torch.manual_seed(M + 3 * N + K)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) * 0.1).to(torch.bfloat16)
    ref = (x.double() @ w.double().t()).cpu()
    z = G.lds_xwt(x, w)
    assert rel_err(z.cpu().numpy(), ref.numpy()) < TOL
    z2, part = G.lds_xwt(x, w, stats=True)
    assert torch.equal(z, z2)
    z16, part16 = G.lds_xwt(x, w, stats=True, out_bf16=True)
    assert torch.equal(z16, z.to(torch.bfloat16)) and torch.equal(part16, part)
    ps = part.double().sum(0).cpu()
    zd = z.double().cpu()
    assert rel_err(ps[0].numpy(), zd.sum(0).numpy()) < 1e-4
    assert rel_err(ps[1].numpy(), (zd * zd).sum(0).numpy()) < 1e-5
    add = torch.randn(M, N + 8, device=cuda)[:, 3:3 + N]
    dst = torch.full((M, N + 16), 7.0, device=cuda)[:, 8:8 + N]
    G.lds_xwt(x, w, out=dst, addend=add)
    assert rel_err(dst.cpu().numpy(), (add.double().cpu() + ref).numpy()) < TOL


def test_lds_xwt_concat_slice_operand(cuda):
    from dgx import gemm as G
    torch.manual_seed(5)
    xcat = torch.randn(2048, 512, device=cuda).to(torch.bfloat16)
    X = xcat[:, 128:256]
    w = torch.randn(512, 128, device=cuda).to(torch.bfloat16)
    ref = (X.double() @ w.double().t()).cpu()
    assert rel_err(G.lds_xwt(X, w).cpu().numpy(), ref.numpy()) < TOL


@pytest.mark.parametrize("R,M,N", [(32768, 1024, 512), (32768, 512, 128), (5000, 128, 64), (1000, 256, 64),
                                   (100, 64, 64), (4099, 128, 128)])
def test_lds_atb_split_k(cuda, R, M, N):
    from dgx import gemm as G
    torch.manual_seed(R + M + N)
    a = torch.randn(R, M, device=cuda).to(torch.bfloat16)
    b = torch.randn(R, N, device=cuda).to(torch.bfloat16)
    ref = (a.double().t() @ b.double()).cpu()
    out = torch.empty(M, N, device=cuda)
    G.lds_atb(a, b, out)
    assert rel_err(out.cpu().numpy(), ref.numpy()) < TOL
    out2 = torch.empty(M, N, device=cuda)
    G.lds_atb(a, b, out2)
    assert torch.equal(out, out2)


def test_lds_atb_strided_concat_operand_and_unstack(cuda):
    from dgx import gemm as G
    torch.manual_seed(9)
    co, c, R = 128, 64, 6000
    dpq = torch.randn(R, 2 * co, device=cuda).to(torch.bfloat16)
    X = torch.randn(R, 512, device=cuda).to(torch.bfloat16)[:, 64:64 + c]
    full = (dpq.double().t() @ X.double()).cpu()
    gw = torch.empty(co, 2 * c, device=cuda)
    G.lds_atb(dpq, X, gw, split_rows=co)
    exp = torch.cat([full[:co], full[co:]], dim=1)
    assert rel_err(gw.cpu().numpy(), exp.numpy()) < TOL


@pytest.mark.parametrize("co,c,stacked", [(64, 64, True), (256, 128, True), (1024, 512, False)])
def test_weight_prep(cuda, co, c, stacked):
    from dgx import gemm as G
    torch.manual_seed(co)
    w = torch.randn(co, 2 * c if stacked else c, 1, 1, device=cuda)
    nt, tn = G.prep_weight(w, co, c, stacked)
    w2 = w.reshape(co, -1)
    exp = torch.cat([w2[:, :c], w2[:, c:]], dim=0) if stacked else w2
    assert torch.equal(nt, exp.to(torch.bfloat16))
    assert torch.equal(tn, exp.t().contiguous().to(torch.bfloat16))


def test_weight_prep_multi(cuda):
    """The batched launch the EdgeConv forward uses equals per-weight prep."""
    from dgx import gemm as G
    torch.manual_seed(5)
    shapes = [(64, 64, True), (128, 64, True), (256, 128, True), (40, 24, False)]
    ws = [torch.randn(co, 2 * c if st else c, 1, 1, device=cuda) for (co, c, st) in shapes]
    got = G.prep_weights([(w, co, c, st) for w, (co, c, st) in zip(ws, shapes)])
    for w, (co, c, st), (nt, tn) in zip(ws, shapes, got):
        ent, etn = G.prep_weight(w, co, c, st)
        assert torch.equal(nt, ent) and torch.equal(tn, etn)


def test_weight_prep_split(cuda):
    """Split form: nt = [W_hi | W_lo] with W_hi = bf16(W), W_lo = bf16(W - W_hi);
    tn stays W_hi^T (the backward operand)."""
    from dgx import gemm as G
    torch.manual_seed(6)
    shapes = [(64, 64, True), (256, 128, True), (1024, 512, False)]
    ws = [torch.randn(co, 2 * c if st else c, 1, 1, device=cuda) for (co, c, st) in shapes]
    got = G.prep_weights([(w, co, c, st, True) for w, (co, c, st) in zip(ws, shapes)])
    for w, (co, c, st), (nt, tn) in zip(ws, shapes, got):
        w2 = w.reshape(co, -1)
        exp = torch.cat([w2[:, :c], w2[:, c:]], dim=0) if st else w2
        hi = exp.to(torch.bfloat16)
        lo = (exp - hi.float()).to(torch.bfloat16)
        assert nt.shape == (exp.shape[0], 2 * c)
        assert torch.equal(nt[:, :c], hi) and torch.equal(nt[:, c:], lo)
        assert torch.equal(tn, hi.t().contiguous())


@pytest.mark.parametrize("M,N,K", [(4096, 128, 64), (3000, 512, 128), (32768, 1024, 512)])
def test_lds_xwt_split_weight(cuda, M, N, K):
    """x16 [W_hi | W_lo]^T with the A tile reused for both halves equals the fp64
    product of the bf16 operand with the 16-significant-bit weight."""
    from dgx import gemm as G
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = torch.randn(N, K, 1, 1, device=cuda) / K ** 0.5
    (nt, _), = G.prep_weights([(w, N, K, False, True)])
    z = G.lds_xwt(x, nt)
    wsplit = nt[:, :K].double() + nt[:, K:].double()
    ref = x.double() @ wsplit.t()
    assert rel_err(z.cpu().numpy(), ref.cpu().numpy()) < TOL
    # and it is closer to the fp32 weight than the hi part alone
    exact = x.double() @ w.reshape(N, K).double().t()
    e_split = float((z.double() - exact).abs().max())
    e_hi = float((G.lds_xwt(x, nt[:, :K].contiguous()).double() - exact).abs().max())
    assert e_split < 0.25 * e_hi


@pytest.mark.parametrize("M,N,K,ta,tb", [(32768, 128, 64, False, True), (32768, 64, 128, False, False),
                                         (130, 70, 33, True, False), (1, 5, 17, False, False),
                                         (256, 512, 32768, True, True), (64, 3, 2048, True, True),
                                         (4096, 1024, 512, False, True), (33000, 200, 77, False, False),
                                         (513, 130, 40960, True, True), (40000, 130, 64, True, False)])
def test_mm32_fp32_mfma(cuda, M, N, K, ta, tb):
    """The parity mode's engine GEMM (dgx_gemm_f32, v_mfma_f32_16x16x4_f32):
    a (M,K) @ b (K,N) for row-major and transposed views read in place,
    ragged edges and the split-K weight-gradient form, against fp64."""
    from dgx import gemm as G
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn((K, M) if ta else (M, K), generator=g)
    b = torch.randn((N, K) if tb else (K, N), generator=g)
    ad, bd = a.to(cuda), b.to(cuda)
    av, bv = (ad.t() if ta else ad), (bd.t() if tb else bd)
    got = G.mm32(av, bv)
    ref = (a.t() if ta else a).double() @ (b.t() if tb else b).double()
    assert rel_err(got.cpu(), ref) < 1e-5
    # accumulate into a column slice of a wider buffer, and the addend form
    wide = torch.randn((M, N + 9), device=cuda)
    base = wide.clone()
    if K < 2048:
        G.mm32(av, bv, out=wide[:, 4:4 + N], accumulate=True)
        assert rel_err(wide[:, 4:4 + N].cpu(), base[:, 4:4 + N].cpu().double() + ref) < 1e-5
        assert torch.equal(wide[:, :4], base[:, :4]) and torch.equal(wide[:, 4 + N:], base[:, 4 + N:])
        add = torch.randn((M, N), device=cuda)
        out = torch.empty((M, N), device=cuda)
        G.mm32(av, bv, out=out, addend=add)
        assert rel_err(out.cpu(), add.cpu().double() + ref) < 1e-5


@pytest.mark.parametrize("M,Co,K", [(32768, 64, 3), (1000, 24, 3), (77, 8, 9)])
def test_smallk_split_weight(cuda, M, Co, K):
    """dgx_gemm_smallk_split_f32 on the reference conv weight (Co, 2K) = [W1 | W2]
    equals the small-K GEMM on the stacked [W1; W2] bit for bit, and fp64."""
    from dgx import gemm as G
    from dgx.edgeconv import split_weight
    g = torch.Generator().manual_seed(M + Co)
    x = torch.randn(M, K, generator=g).to(cuda)
    w = torch.randn(Co, 2 * K, 1, 1, generator=g).to(cuda)
    ref = G.mm_smallk(x, split_weight(w, K, Co))
    out = G.mm_smallk_split(x, w, Co)
    assert torch.equal(out, ref)
    w2 = w.reshape(Co, 2 * K).double()
    exact = x.double() @ torch.cat([w2[:, :K], w2[:, K:]], 0).t()
    assert rel_err(out.cpu(), exact.cpu()) < 1e-6


@pytest.mark.parametrize("M,N,K", [(32768, 64, 128), (32768, 128, 512), (4000, 64, 256), (8192, 128, 256)])
def test_gemm_edge_dz_epilogue(cuda, M, N, K):
    """dgx_gemm_edge_dz_bf16 = the EdgeConv input-gradient GEMM (addend + A W^T)
    followed by dgx_edge_bwd_dz_packed_f32 on its output: the packed dz|slot
    words bit for bit, the BN-backward column partials (other summation order)
    to 1e-5 of their sums."""
    from dgx import _native as nat
    from dgx import bn as bn_
    from dgx import gemm as G
    g = torch.Generator().manual_seed(M + N + K)
    a16 = torch.randn(M, K, generator=g).to(cuda).bfloat16()
    w16 = torch.randn(N, K, generator=g).to(cuda).bfloat16()
    big = torch.randn(M, N + 24, generator=g).to(cuda)
    add = big[:, 8:8 + N]
    ysel = torch.randn(M, N, generator=g).to(cuda)
    arg = torch.randint(0, 20, (M, N), generator=g, dtype=torch.uint8).to(cuda)
    st = bn_.Stats(*(torch.randn(N, generator=g).to(cuda) for _ in range(4)), None, False)
    dz, part, rows = G.lds_xwt_edge_dz(a16, w16, add, ysel, arg, st, 0.2)
    dY = torch.empty(M, N, device=cuda)
    G.lds_xwt(a16, w16, out=dY, addend=add)
    nblk = max(1, min(1024, (M + 63) // 64))
    dz_ref = torch.empty(M, N, device=cuda)
    part_ref = torch.empty(nblk, 2, N, device=cuda)
    L = nat.lib()
    nat.check(L.dgx_edge_bwd_dz_packed_f32(nat.f32(dY), N, nat.f32(ysel), nat.u8(arg), M, N, nat.f32(st.scale),
                                           nat.f32(st.shift), nat.f32(st.mean), nat.f32(st.invstd), 0.2,
                                           nat.f32(dz_ref), nat.f32(part_ref), nblk, nat.stream_of(dY)), "dz")
    torch.cuda.synchronize()
    assert torch.equal(dz.view(torch.int32), dz_ref.view(torch.int32))
    s, s_ref = part.double().sum(0), part_ref.double().sum(0)
    scale = part_ref.double().abs().sum(0)
    assert float(((s - s_ref).abs() / scale.clamp_min(1e-30)).max()) < 1e-5


def test_slab_reduce_multi_matches_single(cuda):
    """dgx_slab_reduce_multi_f32 (the backward's one weight-gradient reduce; the
    4-elements-per-lane path for every job whose columns are a multiple of 4)
    sums every element exactly as dgx_slab_reduce_f32 does: bitwise equal,
    including stacked [W1 | W2] outputs (split) and a strided destination."""
    import ctypes

    from dgx import _native as nat
    L = nat.lib()
    g = torch.Generator(device="cpu").manual_seed(11)
    # (S, rows, cols, split): split == rows is an unstacked output; split < rows
    # puts rows [split, rows) beside rows [0, split) (the [W1 | W2] layout)
    for shapes in ([(16, 1024, 512, 1024), (4, 128, 64, 64), (37, 64, 6, 32)],   # per-job 4-wide / scalar
                   [(16, 130, 66, 130), (3, 20, 3, 10)]):                         # scalar only
        jobs = []
        for S, rows, cols, split in shapes:
            slab = torch.randn(S, rows, cols, generator=g).to(cuda)
            orows, ocols = (rows - split, 2 * cols) if split < rows else (rows, cols)
            out = torch.full((orows, ocols + 4), float("nan"), device=cuda)
            ref = torch.full_like(out, float("nan"))
            nat.check(L.dgx_slab_reduce_f32(nat.f32(slab), S, rows, cols, split, nat.f32(ref), ocols + 4,
                                            nat.stream_of(slab)), "slab single")
            jobs.append((slab, S, rows, cols, split, out, ocols + 4, ref))
        n = len(jobs)
        arr = ctypes.c_void_p * n
        ints = ctypes.c_int * n
        nat.check(L.dgx_slab_reduce_multi_f32(n, arr(*[j[0].data_ptr() for j in jobs]), ints(*[j[1] for j in jobs]),
                                              ints(*[j[2] for j in jobs]), ints(*[j[3] for j in jobs]),
                                              ints(*[j[4] for j in jobs]), arr(*[j[5].data_ptr() for j in jobs]),
                                              (ctypes.c_int64 * n)(*[j[6] for j in jobs]), nat.stream_of(jobs[0][0])),
                  "slab multi")
        torch.cuda.synchronize()
        for j in jobs:
            assert torch.equal(j[5].nan_to_num(7.0), j[7].nan_to_num(7.0))


def test_weight_stack_multi(cuda):
    """dgx_weight_stack_multi_f32 (the fp32 mode's per-pass [W1; W2] builder, one
    launch for every block) equals the reference weight (Co, 2C) split into its
    x_j / x_i halves and stacked: bit-exact, ragged shapes, and >8 jobs rejected."""
    import ctypes

    from dgx import _native as nat
    L = nat.lib()
    g = torch.Generator(device="cpu").manual_seed(12)
    shapes = [(64, 64), (64, 64), (128, 64), (256, 128), (1024, 320), (5, 3), (7, 33)]
    ws = [torch.randn(co, 2 * c, generator=g).to(cuda) for co, c in shapes]
    outs = [torch.full((2 * co, c), float("nan"), device=cuda) for co, c in shapes]
    n = len(shapes)
    arr = ctypes.c_void_p * n
    ints = ctypes.c_int * n
    nat.check(L.dgx_weight_stack_multi_f32(n, arr(*[w.data_ptr() for w in ws]), ints(*[s[0] for s in shapes]),
                                           ints(*[s[1] for s in shapes]), arr(*[o.data_ptr() for o in outs]),
                                           nat.stream_of(ws[0])), "weight stack")
    torch.cuda.synchronize()
    for (co, c), w, o in zip(shapes, ws, outs):
        assert torch.equal(o, torch.cat([w[:, :c], w[:, c:]], 0))
    n9 = 9
    rc = L.dgx_weight_stack_multi_f32(n9, (ctypes.c_void_p * n9)(*([ws[0].data_ptr()] * n9)),
                                      (ctypes.c_int * n9)(*([64] * n9)), (ctypes.c_int * n9)(*([64] * n9)),
                                      (ctypes.c_void_p * n9)(*([outs[0].data_ptr()] * n9)), nat.stream_of(ws[0]))
    assert rc != 0
