"""Optional fp8 GEMMs for the training step (``ModelArgs.fp8`` / ``bench.py --fp8``).

MI355X's matrix cores run OCP fp8 (e4m3fn / e5m2) at twice the bf16 rate; hipBLASLt reaches
1.3-2.3 PFLOP/s on the GPT-2-small projection shapes where the same GEMMs in bf16 reach
0.8-1.3 (``tools/fp8_probe.py``).  Recipe (per-tensor *current* scaling, no amax history):

* forward ``y = x W^T``: x and W quantised to e4m3 (scale = 448 / amax), hipBLASLt fp8 GEMM
  with the bias in its epilogue, bf16 output;
* data gradient ``dx = dy W``: dy quantised to e5m2 (wider range), W^T in e4m3;
* weight gradients stay bf16 x bf16 -> fp32 (our split-K TN kernel), norms / attention /
  softmax / optimizer are unchanged.

Quantisation is one HIP kernel pair per tensor (``csrc/kernels/fp8.hip``: amax, then cast
with the device-side scale), so the step needs no host synchronisation.  This is NOT the
headline configuration (that is bf16 end to end); the bench labels an fp8 run as such.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from .dispatch import shadow

FMAX = {0: 448.0, 1: 57344.0}
_DT = {0: torch.float8_e4m3fn, 1: torch.float8_e5m2}


def quantize_ref(x: torch.Tensor, fmt: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """PyTorch oracle of the quantisation kernel (same fp32 operations, so the same bytes)."""
    amax = x.abs().amax().float().clamp_min(1e-12)
    scale = FMAX[fmt] / amax
    q = (x.float() * scale).to(_DT[fmt])
    return q, (1.0 / scale).reshape(())


def quantize(x: torch.Tensor, fmt: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """(q, inv_scale): q = sat(x * FMAX / amax) in e4m3 (fmt 0) or e5m2 (fmt 1)."""
    if x.is_cuda:
        from . import _ext
        return tuple(_ext.require().fp8_quant(x.contiguous(), fmt))
    return quantize_ref(x, fmt)


def _mm(a8, sa, b8_t, sb, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """bf16 (a8 * sa) @ (b8_t * sb) (+ bias); b8_t is a column-major [K, N] view."""
    if a8.is_cuda:
        return torch._scaled_mm(a8, b8_t, scale_a=sa, scale_b=sb, bias=bias, out_dtype=torch.bfloat16)
    y = (a8.float() * sa) @ (b8_t.float() * sb)
    if bias is not None:
        y = y + bias.float()
    return y.to(torch.bfloat16)


# An fp8 GEMM pays a quantisation pass over its activation operand (amax read + cast read +
# fp8 write, ~2.5 B per element at ~5.5 TB/s) and saves ~0.35 fs per FLOP against bf16
# (0.8-1.3 -> 1.3-2.3 PF/s): it wins when the dimension the operand is multiplied across is
# >~ 640 and clearly from ~2048.  Forward GEMMs quantise x [M, K] and multiply across N =
# W.shape[0]; data-gradient GEMMs quantise dy [M, N] and multiply across K = W.shape[1].
# bench.py --fp8 at GPT-2 small with every projection in fp8 ran 41.8 ms vs 39.5 bf16
# (the lm_head dgrad alone quantises 1.6 G logit gradients).
def min_dim() -> int:
    return int(os.environ.get("DPFS_FP8_MIN_DIM", "2048"))


class Fp8Weight:
    """One step's fp8 copies of a bf16 weight W [N, K]: W in e4m3 for the forward (when N >=
    min_dim()) and a transposed contiguous e4m3 copy for the data gradient (when K >= min_dim();
    hipBLASLt takes the second operand column-major).  Built once per step; the weights change
    every optimizer step."""

    def __init__(self, w: torch.Tensor):
        self.fwd = w.shape[0] >= min_dim()
        self.dgrad = w.shape[1] >= min_dim()
        self.w8, self.s = quantize(w.contiguous(), 0)
        self.wt8 = self.w8.t().contiguous() if self.dgrad else None


def nt(x: torch.Tensor, fw: Fp8Weight, bias: Optional[torch.Tensor] = None, out=None) -> torch.Tensor:
    """y[M, N] = x[M, K] W^T (+ bias) with e4m3 operands, bf16 output."""
    x8, sx = quantize(x, 0)
    bb = shadow(bias, torch.bfloat16) if bias is not None else None
    y = _mm(x8, sx, fw.w8.t(), fw.s, bb).to(x.dtype)     # (bf16 on the GPU: no-op)
    if out is not None:
        out.copy_(y)
        return out
    return y


def nn(dy: torch.Tensor, fw: Fp8Weight, out=None) -> torch.Tensor:
    """dx[M, K] = dy[M, N] W[N, K] with dy in e5m2 and W in e4m3, bf16 output."""
    d8, sd = quantize(dy, 1)
    y = _mm(d8, sd, fw.wt8.t(), fw.s, None).to(dy.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


# ------------------------------------------------------------------ engine hook ------
# The explicit-schedule engines build one Fp8Weight per GEMM weight at the start of a step's
# forward and activate the map for the forward and again for the backward; ops.gemm_select
# looks every weight up here first, so the engines' GEMM call sites stay unchanged.
_active: Optional[dict] = None


def _key(w: torch.Tensor):
    return (w.data_ptr(), tuple(w.shape))


def prepare(weights) -> dict:
    """Fp8Weight for every weight whose dims hipBLASLt's fp8 GEMMs take (multiples of 16) and
    where fp8 pays in at least one direction; the others keep the bf16 path."""
    out = {}
    for w in weights:
        if w is None or w.shape[0] % 16 or w.shape[1] % 16:
            continue
        if w.shape[0] >= min_dim() or w.shape[1] >= min_dim():
            out[_key(w)] = Fp8Weight(w)
    return out


def activate(m: Optional[dict]):
    global _active
    _active = m


def lookup(w: torch.Tensor, dgrad: bool = False) -> Optional[Fp8Weight]:
    """The step's fp8 copy of w if fp8 is on and pays for this use (forward or data grad)."""
    if _active is None or w is None:
        return None
    fw = _active.get(_key(w))
    if fw is None or not (fw.dgrad if dgrad else fw.fwd):
        return None
    return fw
