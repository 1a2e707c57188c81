"""dgx.optim.SGD host logic (no GPU): torch.optim.SGD's argument checks, and a
loud refusal of parameters the HIP kernel cannot take (no silent CPU path)."""
import pytest
import torch


def test_sgd_argument_checks():
    from dgx.optim import SGD
    p = [torch.nn.Parameter(torch.zeros(3))]
    with pytest.raises(ValueError):
        SGD(p, lr=-1.0)
    with pytest.raises(ValueError):
        SGD(p, lr=0.1, momentum=-0.5)
    with pytest.raises(ValueError):
        SGD(p, lr=0.1, weight_decay=-1e-4)
    with pytest.raises(ValueError):
        SGD(p, lr=0.1, momentum=0.0, nesterov=True)
    opt = SGD(p, lr=0.1, momentum=0.9, weight_decay=1e-4)
    assert opt.param_groups[0]["momentum"] == 0.9 and opt.param_groups[0]["nesterov"] is False


def test_sgd_refuses_host_parameters():
    from dgx.optim import SGD
    p = torch.nn.Parameter(torch.zeros(3))
    p.grad = torch.ones(3)
    opt = SGD([p], lr=0.1)
    with pytest.raises(TypeError):
        opt.step()
    q = torch.nn.Parameter(torch.zeros(3))   # no gradient: skipped, nothing launched
    SGD([q], lr=0.1).step()
