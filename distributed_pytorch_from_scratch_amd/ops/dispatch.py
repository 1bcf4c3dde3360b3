"""Device -> kernel-set selection.

``K(t)`` returns the module implementing the kernel API for tensor ``t``: the native HIP
extension for bf16 compute on the GPU, ``ops/fp32_native.py`` (the native fp32 kernel set) for
fp32 compute on the GPU -- both fail loudly if the extension is not built -- and
``ops/reference.py`` (the PyTorch oracle) for CPU tensors.  All three expose the same
function names / signatures.
"""
from __future__ import annotations

import os

import torch

from . import _ext, fp32_native, reference


def K(t: torch.Tensor, dtype: "torch.dtype | None" = None):
    """Kernel set for tensor ``t`` computed in ``dtype`` (default: ``t.dtype``): on the GPU the
    native HIP extension for bf16 work and ``fp32_native`` (fp32-input MFMA GEMMs and flash
    attention + the shared fp32-capable kernels) for fp32 compute -- the reference's default
    training (``train.py`` without ``--bf16``, ``/root/reference/train.py:58-63``); the
    ``reference`` PyTorch oracle on the CPU (and on the GPU only with ``DPFS_FP32_ORACLE=1``,
    an A/B switch)."""
    if t.is_cuda:
        if (dtype or t.dtype) != torch.float32:
            return _ext.require()
        if not _fp32_oracle():
            _ext.require()
            return fp32_native
    return reference


def _fp32_oracle() -> bool:
    return os.environ.get("DPFS_FP32_ORACLE", "0") == "1"


def native_fp32() -> bool:
    """Whether fp32 compute on the GPU runs on the native kernel set (fp32 MFMA GEMMs, fp32
    flash attention) rather than the PyTorch oracle with materialised attention scores."""
    return not _fp32_oracle()


def shadow(p: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Low-precision compute copy of an fp32 master parameter.

    The copy is cached on the parameter and re-cast only when the parameter's version
    counter moved (``load_state_dict``, a torch optimizer step, ``copy_``).  The fused HIP
    Adam (``ops.optim.FusedAdam``) writes the master and the shadow in the same kernel without
    bumping the version, so the steady state costs no cast kernel at all.
    """
    if p.dtype == dtype:
        return p.detach()
    c = getattr(p, "_dpfs_shadow", None)
    if c is not None and c[0] == p._version and c[1].dtype == dtype and c[1].device == p.device \
            and c[1].shape == p.shape:
        return c[1]
    s = p.detach().to(dtype)
    p._dpfs_shadow = (p._version, s)
    return s


def peek_shadow(p: torch.Tensor):
    c = getattr(p, "_dpfs_shadow", None)
    if c is None or c[0] != p._version or c[1].shape != p.shape:
        return None
    return c[1]


_SORT_STREAMS = {}


def emb_sort_ahead(ids: torch.Tensor, vocab_start: int, v_local: int):
    """The deterministic embedding backward's sort (``embedding_bwd_sorted``: the ids' stable
    order and each local vocab row's segment start), issued at the start of the forward on a
    side stream so it runs beside the forward's GEMMs instead of in the backward's tail.
    Returns a handle for :func:`emb_sort_take` (None off the GPU)."""
    if not ids.is_cuda:
        return None
    dev = ids.device
    side = _SORT_STREAMS.get(dev.index)
    if side is None:
        side = _SORT_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    side.wait_stream(cur)                       # the ids are ready
    with torch.cuda.stream(side):
        # deterministic radix sort on our kernels (csrc/kernels/embedding_ce.hip emb_sort)
        perm, seg = _ext.require().emb_sort(ids.view(-1), vocab_start, v_local)
        ev = torch.cuda.Event()
        ev.record(side)
    ids.record_stream(side)
    return perm, seg, ev, side


def emb_sort_take(h):
    """(perm, seg) of an :func:`emb_sort_ahead` handle, ordered before the current stream's
    next work (None, None for no handle)."""
    if h is None:
        return None, None
    perm, seg, ev, side = h
    cur = torch.cuda.current_stream(perm.device)
    cur.wait_event(ev)
    perm.record_stream(cur)                     # (allocated on the side stream, used on this one)
    seg.record_stream(cur)
    return perm, seg
