"""Tensor-parallel linear autograd Functions with the collectives fused in.

The reference composes ``Copy -> F.linear -> +bias`` (column) and
``F.linear -> Reduce -> +bias`` (row) from separate autograd nodes (``models/layers.py:44-100``),
so every column layer's backward all-reduce runs *after* its dgrad and wgrad and the GPU
serialises GEMM -> all-reduce -> GEMM (``SURVEY.md`` §3.3).  Here each parallel linear is one
Function whose backward is ordered for overlap on MI355X:

column-parallel backward (``y = x W^T + b``, ``x`` replicated):
    1. dgrad ``dx = dy W``             (MFMA GEMM, compute stream)
    2. launch ``all_reduce(dx)`` async (RCCL on the process group's own HIP stream)
    3. wgrad ``dW = dy^T x`` (fp32), ``db = colsum(dy)`` while the all-reduce is on the wire
    4. wait on the work handle (stream-ordered, no host sync)

row-parallel forward (``y = sum_r x_r W_r^T + b``): GEMM, in-place all-reduce, bias add
(fused with the residual add by the caller when possible).

Sequence-parallel variants (``sequence_parallel=True``) replace the all-reduce pairs by
all-gather / reduce-scatter over the token dimension (Megatron-SP), the same bytes on the
wire but norms/residuals then run on ``T/tp`` tokens per rank.

All GEMMs go through ``ops.gemm_select`` (``GS.gemm_*``): on GPU they run on our MFMA kernels
(``csrc/kernels/gemm4.hip`` and ``gemm.hip``; the variant is timed once per shape), with
hipBLASLt only when pinned (``DPFS_GEMM_BACKEND=blas``), opted into the timing
(``DPFS_GEMM_LIB=1``) or for a contiguous dimension that is not a multiple of 8; on CPU it is
fp32 torch.  The weight is an fp32 master parameter; the GEMMs read its cached bf16 shadow
(``ops.dispatch.shadow``) and write the weight gradient in fp32.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..ops import gemm_select as GS
from ..ops.dispatch import K, shadow
from . import comm_ops
from . import process_manager as pm


def _compute_w(weight: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    return shadow(weight, x.dtype)


def _bias_grad(k, dy2, bias):
    if bias is None:
        return None
    return k.bias_grad(dy2).to(bias.dtype)


class ColumnParallelLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, sequence_parallel: bool, grad_allreduce: bool):
        k = K(x)
        x_in = x
        if sequence_parallel:
            x = comm_ops.all_gather_rows(x)
        w = _compute_w(weight, x)
        y = GS.gemm_nt(k, x, w, bias)
        # In SP mode keep only the shard; the full activation is re-gathered in backward.
        ctx.save_for_backward(x_in, weight, bias)
        ctx.sp = sequence_parallel
        ctx.ar = grad_allreduce
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, weight, bias = ctx.saved_tensors
        k = K(x2)
        dy2 = dy.reshape(-1, dy.size(-1)).contiguous()
        w = _compute_w(weight, dy2)
        handle = None
        if ctx.sp:
            xg, hg = comm_ops.all_gather_rows(x2, async_op=True)
            dx_full = GS.gemm_nn(k, dy2, w)
            if hg is not None:
                hg.wait()
            dx = comm_ops.reduce_scatter_rows(dx_full)
            x_for_w = xg
        else:
            dx = GS.gemm_nn(k, dy2, w)
            if ctx.ar:
                handle = comm_ops.all_reduce_(dx, async_op=True)
            x_for_w = x2
        dw = k.gemm_tn(dy2, x_for_w).to(weight.dtype) if weight.requires_grad else None
        db = _bias_grad(k, dy2, bias) if (bias is not None and bias.requires_grad) else None
        if handle is not None:
            handle.wait()
        return dx, dw, db, None, None


class RowParallelLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, sequence_parallel: bool, reduce_output: bool):
        k = K(x)
        w = _compute_w(weight, x)
        y = GS.gemm_nt(k, x, w, None)
        if sequence_parallel:
            y = comm_ops.reduce_scatter_rows(y)
        elif reduce_output:
            comm_ops.all_reduce_(y)
        if bias is not None:
            y = k.add_bias_(y, bias)
        ctx.save_for_backward(x, weight, bias)
        ctx.sp = sequence_parallel
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, weight, bias = ctx.saved_tensors
        k = K(x2)
        dy2 = dy.reshape(-1, dy.size(-1)).contiguous()
        db = _bias_grad(k, dy2, bias) if (bias is not None and bias.requires_grad) else None
        if ctx.sp:
            dy2 = comm_ops.all_gather_rows(dy2)
        w = _compute_w(weight, dy2)
        dx = GS.gemm_nn(k, dy2, w)
        dw = k.gemm_tn(dy2, x2).to(weight.dtype) if weight.requires_grad else None
        return dx, dw, db, None, None


def _apply_2d(fn, x, *args):
    # The Functions work on 2-D (tokens, features) tensors; the reshapes stay outside them
    # so their outputs are not custom-Function views (the attention rotates q/k in place).
    if x.dim() == 2:
        return fn.apply(x, *args)
    lead = x.shape[:-1]
    y = fn.apply(x.reshape(-1, x.size(-1)), *args)
    return y.view(*lead, y.size(-1)) if y.size(0) == x.numel() // x.size(-1) else y


def column_parallel_linear(x, weight, bias=None, sequence_parallel=False, grad_allreduce=True):
    return _apply_2d(ColumnParallelLinearFn, x, weight, bias, sequence_parallel, grad_allreduce)


def row_parallel_linear(x, weight, bias=None, sequence_parallel=False, reduce_output=True):
    return _apply_2d(RowParallelLinearFn, x, weight, bias, sequence_parallel, reduce_output)
