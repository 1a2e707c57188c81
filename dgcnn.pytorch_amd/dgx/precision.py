"""GEMM operand precision of the engine.

"fp32" (default): every GEMM on the engine's fp32 MFMA kernel (gemm32.hip,
v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation) or the exact
small-K kernel for the 3-channel layer, and the backward scatter keeps exact
fp32 dz — the parity mode the tests hold to 1e-3 against the reference.
"fp32_split" (opt-in): the fp32 mode with conv5's GEMMs and the EdgeConv
blocks' weight / input gradients as 3-pass split bf16 (x = hi + lo, 16
significant bits per operand: hi.W_hi + hi.W_lo + lo.W_hi, ~2^-16 relative per
product, fp32 sums) and the scatter's dz packed with its slot (18 significant
bits). The EdgeConv forward GEMMs, every kNN input and every BN statistic stay
exact fp32. NOT exact fp32: ~1.5x faster than "fp32" at cfg2.
"bf16": the per-point and conv5 GEMM operands are rounded to bf16, products
accumulate in fp32 and outputs stay fp32 (BASELINE.json cfg2 "bf16"), on the
engine's bf16 MFMA kernels (gemm.hip). kNN distances, BN statistics and every
elementwise stage stay fp32 in every mode.

Set with ``dgx.precision.set("bf16")`` or the environment variable
``DGX_PRECISION=bf16``.

Autocast rule ("kNN upcasts to fp32, GEMMs follow autocast
dtype"), read at each op's entry by ``effective()``:
* ``torch.autocast(dtype=bfloat16)`` -> "bf16": the reference's bf16 autocast
  computes its convs with bf16 operands and fp32 accumulation, as these
  kernels do;
* ``torch.autocast(dtype=float16)`` — the reference's training loop,
  main_partseg_dist.py:221, 253 — -> "fp32_split" (unless the global mode is
  "bf16"): 16 significant bits per operand, finer than fp16's 11, at
  split-bf16 cost. The engine never computes narrower than the reference's
  own AMP step, and its fused chain needs no loss scaling (fp32 range).
kNN, BN statistics and every elementwise stage stay fp32, as autocast keeps
them in the reference.
"""
import contextlib
import functools
import os

import torch

MODES = ("fp32", "fp32_split", "bf16")
_mode = os.environ.get("DGX_PRECISION", "fp32").lower()
if _mode not in MODES:
    raise ValueError(f"DGX_PRECISION must be one of {MODES}, got {_mode!r}")


def get():
    return _mode


def autocast_dtype():
    """torch.float16 / torch.bfloat16 while CUDA autocast to that dtype is
    active on this thread, else None."""
    if not torch.is_autocast_enabled("cuda"):
        return None
    dt = torch.get_autocast_dtype("cuda")
    return dt if dt in (torch.float16, torch.bfloat16) else None


def autocast_reduced():
    """Whether CUDA autocast to fp16 / bf16 is active on this thread."""
    return autocast_dtype() is not None


def effective():
    """The GEMM precision an engine op entered now computes in (one of MODES):
    "bf16" in the bf16 mode or under bf16 autocast; "fp32_split" in that mode
    or under fp16 autocast; else "fp32". Read at the op's entry (the engine's
    autograd Functions run with autocast disabled)."""
    dt = autocast_dtype()
    if _mode == "bf16" or dt is torch.bfloat16:
        return "bf16"
    if _mode == "fp32_split" or dt is torch.float16:
        return "fp32_split"
    return "fp32"


def split():
    """Whether an op entered now runs its fp32 GEMMs as split bf16."""
    return effective() == "fp32_split"


def set(mode):  # noqa: A001 (mirrors get)
    global _mode
    if mode not in MODES:
        raise ValueError(mode)
    _mode = mode


@contextlib.contextmanager
def mode(name):
    """Temporarily run in precision ``name`` (one of MODES)."""
    global _mode
    if name not in MODES:
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
