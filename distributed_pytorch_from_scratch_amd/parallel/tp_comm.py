"""Transport of the tensor-parallel collectives: RCCL or xGMI peer memory.

``DPFS_TP_COMM`` = ``auto`` (default) | ``rccl`` | ``xgmi``.

* ``rccl``: ``torch.distributed`` on the TP group (``nccl`` backend = RCCL on ROCm).
* ``xgmi``: :class:`~.xgmi.XgmiComm` (hand-written peer-memory kernels, all links at once).
* ``auto``: on the first TP all-reduce of the process, every TP rank builds the xGMI
  communicator, checks its result against RCCL on a rank-dependent tensor of the live message
  size, and times both; the group takes xGMI only if it was correct on every rank and faster
  (max over ranks).  Every rank reaches the same decision (it is computed from all-reduced
  numbers), so the call sequence stays identical across the group.

Only the TP group's activation / activation-gradient collectives go through here; DP gradient
buckets, the CE statistics gather and init broadcasts stay on RCCL.
"""
from __future__ import annotations

import os
import sys
import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

from . import process_manager as pm

_decisions: Dict[int, Optional[object]] = {}   # id(tp_group) -> XgmiComm | None (= RCCL)
_info: Dict[int, dict] = {}


def mode() -> str:
    m = os.environ.get("DPFS_TP_COMM", "auto")
    assert m in ("auto", "rccl", "xgmi"), f"DPFS_TP_COMM={m!r}: expected auto | rccl | xgmi"
    return m


def _time_ms(fn, reps: int = 5) -> float:
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0) / reps


def _decide(t: torch.Tensor, p) -> Optional[object]:
    m = mode()
    backend = dist.get_backend(p.tp_group)
    if m == "rccl" or not t.is_cuda or (m == "auto" and backend != "nccl"):
        return None
    from .xgmi import XgmiComm
    g = p.tp_group
    ok = torch.ones(1, device=t.device)
    comm, why = None, ""
    try:
        comm = XgmiComm(g)
    except Exception as e:   # IPC unavailable etc.: the whole group falls back together
        ok.zero_()
        why = f"setup failed: {e}"
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=g)
    if ok.item() == 0:
        if m == "xgmi":
            raise RuntimeError(f"DPFS_TP_COMM=xgmi but the xGMI communicator could not be built ({why})")
        return None
    # correctness on a rank-dependent tensor of the live size, against an fp32 RCCL sum
    gen = torch.Generator(device=t.device).manual_seed(4321 + p.tp_rank)
    x = torch.randn(t.numel(), generator=gen, device=t.device).to(t.dtype)
    ref = x.float()
    dist.all_reduce(ref, group=g)
    y = x.clone()
    comm.all_reduce(y, async_op=False, timeout_s=30.0)
    torch.cuda.synchronize()
    err = (y.float() - ref).abs().max().item()
    tol = 1e-2 * max(1.0, ref.abs().max().item())
    good = comm.error() == 0 and err <= tol
    # Workgroups per call (1024 threads each): every CU that holds one cannot also hold a
    # 2-wave-per-SIMD GEMM block (~250 VGPRs per wave), so the collective must stay narrow to
    # overlap compute (as RCCL's few channels do).  Take the narrowest grid within 10 % of the
    # fastest one measured in isolation.
    grids = (8, 16, 32, 64)
    stats = torch.zeros(2 + len(grids), device=t.device)
    stats[0] = 0.0 if good else 1.0
    if good and m == "auto" and backend == "nccl":
        a = t.detach().clone()
        for i, nb in enumerate(grids):
            comm.set_blocks(nb)
            stats[2 + i] = _time_ms(lambda: comm.all_reduce(a, async_op=False))
        stats[1] = _time_ms(lambda: dist.all_reduce(a, group=g))
        comm.check()
    dist.all_reduce(stats, op=dist.ReduceOp.MAX, group=g)
    bad, t_r = stats[0].item(), stats[1].item()
    best = grids.index(32)
    if not bad and m == "auto" and backend == "nccl":
        times = stats[2:].tolist()
        best = min(i for i, tt in enumerate(times) if tt <= 1.1 * min(times))
    t_x = stats[2 + best].item()
    comm.set_blocks(grids[best])
    use = bad == 0 and (m == "xgmi" or t_x < 0.97 * t_r)
    if m == "xgmi" and bad:
        raise RuntimeError(f"xGMI all-reduce failed validation (max err {err:.3g}, timeout flag {comm.error()})")
    _info[id(g)] = dict(transport="xgmi" if use else "rccl", xgmi_ms=round(t_x, 3), rccl_ms=round(t_r, 3),
                        xgmi_blocks=grids[best], bytes=t.numel() * t.element_size(), valid=not bad)
    if p.global_rank == 0 and os.environ.get("DPFS_QUIET", "0") != "1":
        print(f"[dpfs] TP collectives: {_info[id(g)]}", file=sys.stderr, flush=True)
    return comm if use else None


def _comm(t: torch.Tensor, p):
    if t.dtype not in (torch.bfloat16, torch.float32) or not t.is_cuda:
        return None
    key = id(p.tp_group)
    if key not in _decisions:
        _decisions[key] = _decide(t, p)
    return _decisions[key]


def info() -> Optional[dict]:
    p = pm.pgm
    return None if p is None else _info.get(id(p.tp_group))


def all_reduce(t: torch.Tensor, async_op: bool = True):
    """SUM over the TP group, in place.  Returns a work handle (``wait()``) or None."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        return None
    c = _comm(t, p)
    if c is None:
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=p.tp_group, async_op=async_op)
    return c.all_reduce(t, async_op=async_op)


def reduce_scatter(out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
    """out = rank-th of tp_size equal row blocks of SUM(inp) over the TP group."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        out.copy_(inp.view_as(out))
        return None
    c = _comm(inp, p)
    if c is None or inp.numel() * inp.element_size() > c.cap or inp.numel() % (8 * p.tp_size):
        return dist.reduce_scatter_tensor(out, inp, group=p.tp_group, async_op=async_op)
    return c.reduce_scatter(out, inp, async_op=async_op)


def all_gather(out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
    """out = concatenation (rank order, dim 0) of inp over the TP group."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        out.copy_(inp.view_as(out))
        return None
    c = _comm(inp, p)
    if c is None or inp.numel() * inp.element_size() > c.cap or inp.numel() % 8:
        return dist.all_gather_into_tensor(out, inp, group=p.tp_group, async_op=async_op)
    return c.all_gather(out, inp, async_op=async_op)


def staging(slot: int, shape, dtype: torch.dtype) -> Optional[torch.Tensor]:
    """Output buffer for a GEMM whose result feeds the next TP all-reduce / reduce-scatter:
    a view of the xGMI communicator's staging slot ``slot`` (then the collective skips its
    copy-in), or None when the group runs on RCCL, has not chosen yet, or it does not fit.
    Use one slot per in-flight chunk; a slot may be rewritten once the collective that read
    it has been waited."""
    p = pm.pgm
    if p is None or p.tp_size == 1 or os.environ.get("DPFS_XGMI_STAGING", "1") == "0":
        return None
    c = _decisions.get(id(p.tp_group))
    if c is None:
        return None
    return c.staging(slot, shape, dtype)


def check():
    """Raise if any xGMI call of this process timed out (cheap: one host-mapped word)."""
    p = pm.pgm
    if p is None:
        return
    c = _decisions.get(id(p.tp_group))
    if c is not None:
        c.check()
