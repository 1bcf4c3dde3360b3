"""Autograd Functions over the kernel API (HIP on GPU, ``reference`` on CPU).

Each Function is a thin, allocation-aware wrapper: the forward saves exactly what the
hand-written backward kernel needs (e.g. RMSNorm saves ``rstd`` per row instead of
autograd's 7 intermediate tensors, attention saves the log-sum-exp instead of the
``(B,H,T,T)`` probabilities of ``models/model.py:73-77``).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .dispatch import K


def _2d(x: torch.Tensor) -> torch.Tensor:
    return x.reshape(-1, x.size(-1))


# ---------------------------------------------------------------------------- RMSNorm ----

class RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps: float):
        shp = x.shape
        x2 = _2d(x).contiguous()
        y, rstd = K(x).rmsnorm_fwd(x2, weight, eps)
        ctx.save_for_backward(x2, weight, rstd)
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        dx, dw = K(x2).rmsnorm_bwd(_2d(dy).contiguous(), x2, w, rstd)
        return dx.view(dy.shape), dw.to(w.dtype), None


def rms_norm(x, weight, eps: float = 1e-5):
    return RMSNormFn.apply(x, weight, eps)


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps: float):
        shp = x.shape
        x2 = _2d(x).contiguous()
        y, mean, rstd = K(x).layernorm_fwd(x2, weight, bias, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = K(x2).layernorm_bwd(_2d(dy).contiguous(), x2, w, mean, rstd)
        return dx.view(dy.shape), dw.to(w.dtype), db.to(w.dtype), None


def layer_norm(x, weight, bias, eps: float = 1e-5):
    return LayerNormFn.apply(x, weight, bias, eps)


# ------------------------------------------------------------------------- SwiGLU ----

class SwiGLUFn(torch.autograd.Function):
    """h = silu(gu[..., :F]) * gu[..., F:] for the fused gate|up GEMM output."""

    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        return K(gu).swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        return K(gu).swiglu_bwd(dh.contiguous(), gu)


def swiglu(gu):
    return SwiGLUFn.apply(gu)


# ---------------------------------------------------------------------- Attention ----

class CausalSelfAttentionFn(torch.autograd.Function):
    """RoPE + causal flash attention on a packed ``qkv[B*T, (hq+hk+hv)*hd]`` GEMM output.

    Forward rotates q and k in place (the buffer is a fresh GEMM output nobody else saved),
    runs the flash-attention forward (O(T) memory, LSE saved), returns ``o[B*T, hq*hd]``.
    Backward runs the flash backward into one packed ``dqkv`` buffer with the inverse rotation
    fused into the dq/dk stores, so the QKV dgrad GEMM consumes it directly.
    """

    @staticmethod
    def forward(ctx, qkv, positions, rope_table, B: int, T: int, hq: int, hkv: int, hd: int,
                causal: bool):
        k_ = K(qkv)
        if rope_table is not None:
            k_.rope_(qkv, positions, rope_table, hq + hkv, hd, False)
        q, k, v = _split_qkv(qkv, B, T, hq, hkv, hd)
        scale = 1.0 / math.sqrt(hd)
        o, lse = k_.attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(qkv, o, lse, positions, rope_table)
        ctx.meta = (B, T, hq, hkv, hd, causal, scale)
        return o.view(B * T, hq * hd)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, positions, rope_table = ctx.saved_tensors
        B, T, hq, hkv, hd, causal, scale = ctx.meta
        k_ = K(qkv)
        q, k, v = _split_qkv(qkv, B, T, hq, hkv, hd)
        do4 = do.contiguous().view(B, T, hq, hd)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = _split_qkv(dqkv, B, T, hq, hkv, hd)
        rp = positions.reshape(-1).long().contiguous() if rope_table is not None else None
        k_.attn_bwd(do4, q, k, v, o, lse, scale, causal, dq, dk, dv, rp, rope_table)  # + inverse RoPE
        return dqkv, None, None, None, None, None, None, None, None


def _split_qkv(qkv, B, T, hq, hkv, hd):
    q = qkv[:, : hq * hd].view(B, T, hq, hd)
    k = qkv[:, hq * hd:(hq + hkv) * hd].view(B, T, hkv, hd)
    v = qkv[:, (hq + hkv) * hd:(hq + 2 * hkv) * hd].view(B, T, hkv, hd)
    return q, k, v


def causal_self_attention(qkv, positions, rope_table, B, T, hq, hkv, hd, causal=True):
    return CausalSelfAttentionFn.apply(qkv, positions, rope_table, B, T, hq, hkv, hd, causal)
