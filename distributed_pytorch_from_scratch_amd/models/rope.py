"""Rotary position embedding helpers with the reference's public API.

Parity: ``models/model.py:17-46`` (``rotate_half``, ``apply_rotary_pos_emb``, ``get_cos_sin``)
— same rotate-half convention, the same fp32 CPU computation of the inverse frequencies, and
full-width ``(seq, head_dim)`` cos/sin tables (both halves equal), so external code written
against the reference keeps working.  ``DTYPE`` / ``DEVICE`` env vars are honoured as in the
reference (``SURVEY.md`` §2.6), but only when no explicit ``dtype`` / ``device`` is passed.

The training path never materialises these tables per layer: the hot path uses one
half-width ``[cos | sin]`` fp32 table (``ops.reference.rope_table``) that the HIP kernels
index by position id (fused into the QKV GEMM epilogue forward and into the attention
backward stores).  These helpers are the eager/oracle form.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch


def rotate_half(x: torch.Tensor) -> torch.Tensor:
    """[x1, x2] -> [-x2, x1] over the last dim."""
    h = x.shape[-1] // 2
    return torch.cat((x[..., h:].neg(), x[..., :h]), dim=-1)


def apply_rotary_pos_emb(q: torch.Tensor, k: torch.Tensor, cos: torch.Tensor,
                         sin: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """q, k: ``(b, heads, t, hd)``; cos, sin: ``(b, t, hd)`` (gathered by position id)."""
    if cos.ndim != 3 or sin.ndim != 3:
        raise ValueError(f"cos/sin must be (batch, seq, head_dim), got {tuple(cos.shape)} / {tuple(sin.shape)}")
    c, s = cos.unsqueeze(1), sin.unsqueeze(1)
    return q * c + rotate_half(q) * s, k * c + rotate_half(k) * s


def _env_dtype() -> torch.dtype:
    return torch.bfloat16 if os.getenv("DTYPE", "float32") == "bfloat16" else torch.float32


def _env_device() -> torch.device:
    want_cuda = os.getenv("DEVICE", "cuda") == "cuda"
    return torch.device("cuda") if want_cuda and torch.cuda.is_available() else torch.device("cpu")


def get_cos_sin(seq_length: int, head_dim: int, base: float, dtype: Optional[torch.dtype] = None,
                device: Optional[torch.device] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Full-width ``(seq_length, head_dim)`` cos and sin tables (each half repeated)."""
    if head_dim % 2:
        raise ValueError("head_dim must be even")
    dtype = dtype or _env_dtype()
    device = torch.device(device) if device is not None else _env_device()
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))  # CPU fp32
    ang = torch.arange(seq_length, device=device).float().unsqueeze(1) * inv.to(device)
    return ang.cos().to(dtype).repeat(1, 2), ang.sin().to(dtype).repeat(1, 2)


def half_table_from_full(cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Convert reference-style full tables to the kernels' fp32 ``[cos | sin]`` half table."""
    h = cos.shape[-1] // 2
    return torch.cat([cos[..., :h].float(), sin[..., :h].float()], dim=-1).contiguous()
