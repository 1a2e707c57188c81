"""torch.optim.SGD with its update in one HIP launch (libdgx.so dgx_sgd_step_f32).

Same constructor, hyper-parameters, state (``state[p]["momentum_buffer"]``) and
update as ``torch.optim.SGD`` (torch/optim/sgd.py), for fp32 parameters on a
ROCm device. torch's fused / foreach forms split a parameter list into
65536-element chunks with one workgroup each — a DGCNN's ~0.6 M parameters
run on ~22 workgroups, ~28 us per step at cfg2; here the whole list is one
grid-stride launch (48 tensors per launch). The training scripts of the
reference construct torch.optim.SGD / Adam (main_partseg.py); this class is a
drop-in for the SGD case. Capturable in a HIP graph once the momentum buffers
exist (after the first step), with FIXED hyper-parameters: lr, momentum,
dampening and weight decay are kernel arguments, so a scheduler's change to
them reaches eager steps but not an already captured graph (recapture after
changing them). Parameters of one group may live on several devices: each
launch takes one device's tensors."""
import ctypes

import torch

from . import _native as nat

_MAX = 48


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, *,
                 maximize=False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov, maximize=maximize))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = nat.lib()
        for group in self.param_groups:
            mom = float(group["momentum"])
            # (first step of a buffer, parameter) lists: torch sets buf = d_p on a
            # parameter's first step, momentum * buf + (1 - dampening) * d_p after
            jobs = {}   # (first step, device) -> [(param, buffer)]: one launch per device
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_cuda:
                    raise TypeError("dgx.optim.SGD: fp32 parameters on a ROCm device expected")
                if p.grad.is_sparse:
                    raise RuntimeError("dgx.optim.SGD: sparse gradients are not supported")
                if not (p.is_contiguous() and p.grad.is_contiguous()):
                    raise RuntimeError("dgx.optim.SGD: contiguous parameters and gradients expected")
                first = False
                buf = None
                if mom != 0.0:
                    st = self.state[p]
                    buf = st.get("momentum_buffer")
                    if buf is None:
                        buf = torch.empty_like(p, memory_format=torch.contiguous_format)
                        st["momentum_buffer"] = buf
                        first = True
                jobs.setdefault((first, p.device), []).append((p, buf))
            for (first, dev), lst in jobs.items():
                for c in range(0, len(lst), _MAX):
                    chunk = lst[c:c + _MAX]
                    n = len(chunk)
                    ps = (ctypes.c_void_p * n)(*[p.data_ptr() for p, _ in chunk])
                    gs = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p, _ in chunk])
                    ms = (ctypes.c_void_p * n)(*[(b.data_ptr() if b is not None else 0) for _, b in chunk])
                    ns = (ctypes.c_int64 * n)(*[p.numel() for p, _ in chunk])
                    with torch.cuda.device(dev):
                        nat.check(lib.dgx_sgd_step_f32(n, ps, gs, ms if mom != 0.0 else None, ns, float(group["lr"]),
                                                       float(group["weight_decay"]), mom, float(group["dampening"]),
                                                       int(group["nesterov"]), int(group["maximize"]), int(first),
                                                       nat.stream_of(chunk[0][0])), "sgd step")
        return loss
