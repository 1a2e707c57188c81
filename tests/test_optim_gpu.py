"""dgx.optim.SGD (one-launch multi-tensor update, csrc/optim.hip) against
torch.optim.SGD's single-tensor form on the same parameters and gradients:
three steps (the first initialises the momentum buffers), every hyper-parameter
combination the bench and the reference's scripts use plus Nesterov /
dampening / maximize, 60 tensors of odd sizes (two launches of <= 48)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kw", [dict(lr=0.1, momentum=0.9, weight_decay=1e-4),
                                dict(lr=0.05),
                                dict(lr=0.1, momentum=0.9, nesterov=True, weight_decay=5e-4),
                                dict(lr=0.2, momentum=0.5, dampening=0.3, maximize=True)])
def test_sgd_matches_torch(cuda, kw):
    from dgx.optim import SGD
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(int(torch.randint(1, 700, (1,), generator=g)),) for _ in range(57)] + [(64, 6), (1024, 512), (3,)]
    ref = [torch.randn(s, generator=g).to(cuda) for s in shapes]
    ours = [t.clone() for t in ref]
    for t in ref + ours:
        t.requires_grad_(True)
    o_ref = torch.optim.SGD(ref, foreach=False, **kw)
    o_dgx = SGD(ours, **kw)
    for _ in range(3):
        for a, b in zip(ref, ours):
            gr = torch.randn(a.shape, generator=g).to(cuda)
            a.grad = gr.clone()
            b.grad = gr.clone()
        o_ref.step()
        o_dgx.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, ours):
        err = ((a - b).abs().max() / a.abs().max().clamp_min(1e-30)).item()
        assert err < 1e-6, err
        if kw.get("momentum", 0):
            mb = o_ref.state[a]["momentum_buffer"]
            err_m = ((mb - o_dgx.state[b]["momentum_buffer"]).abs().max() / mb.abs().max()).item()
            assert err_m < 1e-6, err_m
