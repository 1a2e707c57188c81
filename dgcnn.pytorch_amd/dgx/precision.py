"""GEMM operand precision of the engine.

"fp32" (default): every GEMM on the engine's fp32 MFMA kernel (gemm32.hip,
v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation) or the exact
small-K kernel for the 3-channel layer — the parity mode the tests hold to
1e-3 against the reference.
"bf16": the per-point and conv5 GEMM operands are rounded to bf16, products
accumulate in fp32 and outputs stay fp32 (BASELINE.json cfg2 "bf16"), on the
engine's bf16 MFMA kernels (gemm.hip). kNN distances, BN statistics and every
elementwise stage stay fp32 either way.

Set with ``dgx.precision.set("bf16")`` or the environment variable
``DGX_PRECISION=bf16``.

Autocast rule ("kNN upcasts to fp32, GEMMs follow autocast
dtype"): under ``torch.autocast("cuda", dtype=float16|bfloat16)`` — the
reference's training loop, main_partseg_dist.py:221, 253 — the engine's GEMMs
take their reduced-precision path, whatever the global mode says
(``effective()``). The engine's reduced-precision kernels are bf16 MFMA
(gfx950's 16-bit MFMA rate is the same for fp16 and bf16; bf16 keeps fp32's
exponent range, so no loss scaling is needed inside the fused chain); fp16
autocast therefore routes to them too. kNN, BN statistics and every
elementwise stage stay fp32, as autocast keeps them in the reference.
"""
import contextlib
import functools
import os

import torch

_mode = os.environ.get("DGX_PRECISION", "fp32").lower()
if _mode not in ("fp32", "bf16"):
    raise ValueError(f"DGX_PRECISION must be fp32 or bf16, got {_mode!r}")


def get():
    return _mode


def autocast_reduced():
    """Whether CUDA autocast to fp16 / bf16 is active on this thread."""
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") in (torch.float16, torch.bfloat16)


def effective():
    """The GEMM precision an engine op entered now computes in: "bf16" in the
    bf16 mode or under fp16/bf16 autocast, else "fp32". Read at the op's
    entry (the engine's autograd Functions run with autocast disabled)."""
    return "bf16" if (_mode == "bf16" or autocast_reduced()) else "fp32"


def set(mode):  # noqa: A001 (mirrors get)
    global _mode
    if mode not in ("fp32", "bf16"):
        raise ValueError(mode)
    _mode = mode


@contextlib.contextmanager
def mode(name):
    """Temporarily run in precision ``name`` ("fp32" / "bf16")."""
    global _mode
    if name not in ("fp32", "bf16"):
        raise ValueError(name)
    prev, _mode = _mode, name
    try:
        yield
    finally:
        _mode = prev


def operand(t):
    """GEMM operand in the current precision (bf16 copies are dense)."""
    return t.to(torch.bfloat16) if _mode == "bf16" else t


def mm(a, b, out=None, accumulate=False):
    """a @ b (fp32 output) on the engine's GEMMs in the current precision:
    fp32 MFMA (dgx.gemm.mm32) or bf16 operands with fp32 accumulation
    (dgx.gemm.mm16). Transposed views are read in place. ``accumulate``:
    out += a @ b."""
    from . import gemm
    if _mode == "bf16":
        return gemm.mm16(a, b, out=out, accumulate=accumulate)
    return gemm.mm32(a, b, out=out, accumulate=accumulate)


def no_autocast(fn):
    """Run an autograd.Function's forward/backward with CUDA autocast disabled.

    The reference's DDP script runs the model under torch.cuda.amp.autocast
    (main_partseg_dist.py:253). Inside the engine's Functions every product
    must come back in the dtype its consumer kernel is built for, so autocast
    must not re-type a torch.mm there; each op computes in the precision
    ``effective()`` gave at its entry, on fp32 inputs (each Function casts its
    input)."""
    @functools.wraps(fn)
    def wrapped(*args, **kwargs):
        if torch.is_autocast_enabled("cuda"):
            with torch.autocast("cuda", enabled=False):
                return fn(*args, **kwargs)
        return fn(*args, **kwargs)
    return wrapped
