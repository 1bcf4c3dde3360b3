"""The fp32 kernel set on the GPU (the reference's default training mode).

The reference trains in fp32 unless ``--bf16`` is passed (``/root/reference/train.py:58-63``:
``DTYPE=float32``, no autocast).  Here that mode runs on native gfx950 kernels too:

* GEMMs: ``gemm_f32`` -- fp32-input MFMA (``v_mfma_f32_32x32x2_f32``, exact fp32 at the vector
  rate; ``csrc/kernels/fp32.hip``) in the three layouts of a parallel linear, bias in the
  epilogue, accumulating weight gradients in place;
* attention: ``attn_fwd_f32`` / ``attn_bwd_f32`` -- causal flash attention on the same fp32
  MFMAs (log-sum-exp saved, inverse RoPE and the QKV bias gradient in the backward);
* norms, residual adds, RoPE, SwiGLU, embedding, cross-entropy, column sums and Adam: the
  same HIP kernels as bf16 (they are templated on the storage type, fp32 accumulate).

It exposes the ``ops/reference.py`` API (``ops.dispatch.K`` returns it for fp32 compute on
the GPU).  The fused epilogues that only exist as bf16 MFMA kernels (SwiGLU in the gate|up
GEMM, SwiGLU backward in the down-projection dgrad, the one-pass TP-1 cross-entropy) decline
with ``None`` and the engines run their separate-kernel forms.  The single-token decode
kernels are bf16-only; an fp32 decode runs the reference's tensor ops.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _ext, reference

DIRECT = True   # ops.gemm_select: call the kernels directly (no per-shape candidate timing)


def _C():
    return _ext.require()


def gemm_nt(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None, rope_pos=None, rope_tab=None,
            rope_heads: int = 0, rope_hd: int = 0, out: Optional[torch.Tensor] = None, variant: int = 0):
    c = _C().gemm_f32(a, b, 0, bias, out)
    if rope_pos is not None and rope_heads > 0:
        _C().rope_(c, rope_pos, rope_tab, rope_heads, rope_hd, False)
    return c


def gemm_nn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, variant: int = 0):
    return _C().gemm_f32(a, b, 1, None, out)


def gemm_tn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
            variant: int = 0):
    return _C().gemm_f32(a, b, 2, None, out, bool(accumulate and out is not None))


def gemm_tn2(a0, b0, a1, b1, out=None, accumulate: bool = False):
    c = gemm_tn(a0, b0, out, accumulate)
    return gemm_tn(a1, b1, c, True)


def gemm_nt_swiglu(a, b, bias=None):
    return None      # no fp32 fused-epilogue kernel: gemm_nt + swiglu_fwd


def gemm_nn_swiglu_bwd(dy, w, gu, dbias=None, perm: bool = True):
    return None      # gemm_nn + swiglu_bwd


def ce_fused(logits, targets, gscale, vocab_start, vocab_valid, dbias=None):
    return None      # the one-pass CE kernel reads bf16 logits: stats + backward pass


def attn_supported(hd: int) -> bool:
    """head_dim 32 / 64 / 128 (the presets' 64 and 128 included); others run the oracle."""
    return hd in (32, 64, 128)


def attn_fwd(q, k, v, scale: float, causal: bool = True, impl: int = 0):
    if not attn_supported(q.size(-1)):
        return reference.attn_fwd(q, k, v, scale, causal)
    return _C().attn_fwd_f32(q, k, v, float(scale), bool(causal))


def attn_bwd(do, q, k, v, o, lse, scale: float, causal: bool, dq_out, dk_out, dv_out, rope_pos=None,
             rope_tab=None, dbias=None, impl: int = 0):
    if not attn_supported(q.size(-1)):
        return reference.attn_bwd(do, q, k, v, o, lse, scale, causal, dq_out, dk_out, dv_out, rope_pos, rope_tab,
                                  dbias=dbias)
    return _C().attn_bwd_f32(do, q, k, v, o, lse, float(scale), bool(causal), dq_out, dk_out, dv_out,
                             rope_pos, rope_tab, dbias)


def gemv_nt_ok(x, w, swiglu: bool = False) -> bool:
    return False


# single-token decode (models/generation.py): bf16 kernels only; fp32 decode on tensor ops
attn_decode = reference.attn_decode
kv_append = reference.kv_append
rope_append = reference.rope_append
step_advance = reference.step_advance
gemv_nt = reference.gemv_nt


def __getattr__(name):
    # every other op (norms, RoPE, SwiGLU, embedding, CE, column sums, Adam, the embedding sort,
    # the CE bookkeeping): the native kernel, which takes fp32 storage as well as bf16
    return getattr(_ext.require(), name)
