"""conv5's BatchNorm + LeakyReLU passes in the fp32 mode (the autograd of
dgcnn.py:74-78, 102 through BatchNorm2d train mode) on the 128-point LDS tiles:

* dgx_pointconv_bwd_split_f32 pass 0 gives the same per-channel (sum d,
  sum d*zhat) as the 64-point-tile pass dgx_pointconv_bwd_f32 (1e-6: only the
  fp32 partial-row grouping differs);
* pass 1, given the same c0 / c1, writes bitwise the split-bf16 planes that
  dgx_pointconv_input_grad (fp32 dZ) + dgx_split_bf16 produce;
* dgx_pointconv_apply_f32 on dense rows (the tile kernel) equals the strided
  path bitwise."""

import pytest
import torch

from dgx import _native as nat

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,N,C", [(4, 1024, 1024), (3, 1000, 68), (2, 130, 256)])
def test_pointconv_split_matches_unfused(cuda, B, N, C):
    L = nat.lib()
    g = torch.Generator(device="cpu").manual_seed(N + C)
    M = B * N
    dout = torch.randn(B, C, N, generator=g).to(cuda)
    Z = torch.randn(M, C, generator=g).to(cuda)
    scale = torch.randn(C, generator=g).to(cuda)
    shift = torch.randn(C, generator=g).to(cuda)
    mean = torch.randn(C, generator=g).to(cuda) * 0.1
    invstd = torch.rand(C, generator=g).to(cuda) + 0.5
    stream = nat.stream_of(Z)
    # unfused: dz + partials, finalize, fp32 dZ, split
    rows0 = L.dgx_pointconv_bwd_rows(B, N)
    dz = torch.empty(M, C, device=cuda)
    p0 = torch.empty(rows0, 2, C, device=cuda)
    nat.check(L.dgx_pointconv_bwd_f32(nat.f32(dout), nat.f32(Z), C, B, N, C, nat.f32(scale), nat.f32(shift),
                                      nat.f32(mean), nat.f32(invstd), 0.2, nat.f32(dz), nat.f32(p0), stream), "bwd")
    cs = [torch.empty(C, device=cuda) for _ in range(4)]
    nat.check(L.dgx_bn_bwd_finalize_f32(nat.f32(p0), rows0, C, float(M), nat.f32(scale), nat.f32(mean),
                                        nat.f32(invstd), *(nat.f32(t) for t in cs), 0, stream), "finalize")
    dZ = torch.empty(M, C, device=cuda)
    nat.check(L.dgx_pointconv_input_grad(nat.f32(dz), nat.f32(Z), C, M, C, nat.f32(scale), nat.f32(cs[2]),
                                         nat.f32(cs[3]), nat.f32(dZ), 0, stream), "dZ")
    hi0 = torch.empty(M, C, device=cuda, dtype=torch.bfloat16)
    lo0 = torch.empty_like(hi0)
    nat.check(L.dgx_split_bf16(nat.f32(dZ), C, M, C, nat.bf16(hi0), nat.bf16(lo0), C, stream), "split")
    # fused: stats pass, then dZ straight into the planes with the same c0 / c1
    rows1 = L.dgx_pointconv_bf16_rows(B, N)
    p1 = torch.empty(rows1, 2, C, device=cuda)
    nat.check(L.dgx_pointconv_bwd_split_f32(nat.f32(dout), nat.f32(Z), B, N, C, nat.f32(scale), nat.f32(shift),
                                            nat.f32(mean), nat.f32(invstd), 0.2, None, None, nat.f32(p1), None, None,
                                            0, stream), "stats")
    hi1 = torch.empty_like(hi0)
    lo1 = torch.empty_like(hi0)
    nat.check(L.dgx_pointconv_bwd_split_f32(nat.f32(dout), nat.f32(Z), B, N, C, nat.f32(scale), nat.f32(shift),
                                            None, None, 0.2, nat.f32(cs[2]), nat.f32(cs[3]), None, nat.bf16(hi1),
                                            nat.bf16(lo1), 1, stream), "split dZ")
    torch.cuda.synchronize()
    s0, s1 = p0.double().sum(0), p1.double().sum(0)
    assert ((s0 - s1).abs().max() / s0.abs().max()).item() < 1e-6
    assert torch.equal(hi0, hi1) and torch.equal(lo0, lo1)
    # forward apply: tile kernel (dense Z) vs the strided path
    out_t = torch.empty(B, C, N, device=cuda)
    nat.check(L.dgx_pointconv_apply_f32(nat.f32(Z), C, B, N, C, nat.f32(scale), nat.f32(shift), 0.2, nat.f32(out_t),
                                        stream), "apply tile")
    Zs = torch.zeros(M, C + 4, device=cuda)
    Zs[:, :C] = Z
    out_s = torch.empty_like(out_t)
    nat.check(L.dgx_pointconv_apply_f32(nat.f32(Zs), C + 4, B, N, C, nat.f32(scale), nat.f32(shift), 0.2,
                                        nat.f32(out_s), stream), "apply strided")
    torch.cuda.synchronize()
    assert torch.equal(out_t, out_s)
