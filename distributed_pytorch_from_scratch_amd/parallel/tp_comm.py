"""Transport of the tensor-parallel collectives: RCCL or xGMI peer memory.

``DPFS_TP_COMM`` = ``auto`` (default) | ``rccl`` | ``xgmi``.

* ``rccl``: ``torch.distributed`` on the TP group (``nccl`` backend = RCCL on ROCm).
* ``xgmi``: :class:`~.xgmi.XgmiComm` (hand-written peer-memory kernels, all links at once).
* ``auto``: on the first TP collective of the process, every TP rank builds the xGMI
  communicator and, for each of all-reduce, reduce-scatter and all-gather separately, checks
  its result against RCCL on a rank-dependent tensor of the live message size and times both
  (xGMI at several grid widths); an op goes to xGMI only if it was correct on every rank and
  faster (max over ranks).  Every rank reaches the same decisions (they are computed from
  all-reduced numbers), so the call sequence stays identical across the group.

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

_decisions: Dict[int, Optional["_Choice"]] = {}   # id(tp_group) -> per-op transport (None = RCCL)
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


_OPS = ("all_reduce", "reduce_scatter", "all_gather")
_GRIDS = (8, 16, 32, 64)


class _Choice:
    """The group's communicator and which ops run on it (the rest stay on RCCL)."""

    def __init__(self, comm, use: Dict[str, bool]):
        self.comm, self.use = comm, use


def _xgmi_op(comm, op: str, x: torch.Tensor, part: torch.Tensor, gathered: torch.Tensor, timeout_s=None):
    if op == "all_reduce":
        comm.all_reduce(x, async_op=False, timeout_s=timeout_s)
    elif op == "reduce_scatter":
        comm.reduce_scatter(part, x, async_op=False, timeout_s=timeout_s)
    else:
        comm.all_gather(gathered, part, async_op=False, timeout_s=timeout_s)


def _rccl_op(op: str, g, x, part, gathered):
    if op == "all_reduce":
        dist.all_reduce(x, group=g)
    elif op == "reduce_scatter":
        dist.reduce_scatter_tensor(part, x, group=g)
    else:
        dist.all_gather_into_tensor(gathered, part, group=g)


def _decide(t: torch.Tensor, p) -> Optional[_Choice]:
    m = mode()
    backend = dist.get_backend(p.tp_group)
    if m == "rccl" or not t.is_cuda or (m == "auto" and backend != "nccl"):
        return None
    from .xgmi import XgmiComm
    g = p.tp_group
    W, r = p.tp_size, p.tp_rank
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
    # Correctness of every op on a rank-dependent tensor of the live size, against fp32 sums
    # (RCCL / gloo all-reduce only: the all-gather oracle is a zero-padded sum, exact).
    n = min(t.numel(), comm._max_elems(t))
    n = max(8 * W, n - n % (8 * W))
    gen = torch.Generator(device=t.device).manual_seed(4321 + r)
    x = torch.randn(n, generator=gen, device=t.device).to(t.dtype)
    ref = x.float()
    dist.all_reduce(ref, group=g)
    mine = x.view(W, -1)[r]
    pad = torch.zeros(W, n // W, device=t.device)
    pad[r] = mine.float()
    dist.all_reduce(pad, group=g)
    tol = 1e-2 * max(1.0, ref.abs().max().item())
    y, part, gathered = x.clone(), torch.empty_like(mine), torch.empty_like(x)
    _xgmi_op(comm, "all_reduce", y, None, None, 30.0)
    _xgmi_op(comm, "reduce_scatter", x, part, None, 30.0)
    _xgmi_op(comm, "all_gather", None, mine, gathered, 30.0)
    torch.cuda.synchronize()
    errs = [(y.float() - ref).abs().max().item(), (part.float() - ref.view(W, -1)[r]).abs().max().item(),
            (gathered.float() - pad.view(-1)).abs().max().item()]
    good = [comm.error() == 0 and errs[0] <= tol, comm.error() == 0 and errs[1] <= tol,
            comm.error() == 0 and errs[2] == 0.0]
    # Workgroups per call (1024 threads each): every CU that holds one cannot also hold a
    # 2-wave-per-SIMD GEMM block (~250 VGPRs per wave), so a collective must stay narrow to
    # overlap compute (as RCCL's few channels do).  Per op, take the narrowest grid within
    # 10 % of the fastest one measured in isolation.
    G = len(_GRIDS)
    stats = torch.zeros(3 + 3 + 3 * G, device=t.device)   # bad[3], rccl_ms[3], xgmi_ms[3][G]
    for i in range(3):
        stats[i] = 0.0 if good[i] else 1.0
    timed = all(good) and m == "auto" and backend == "nccl"
    if timed:
        a, ap, ag = t.detach().reshape(-1)[:n].clone(), torch.empty_like(mine), torch.empty_like(x)
        for i, op in enumerate(_OPS):
            for j, nb in enumerate(_GRIDS):
                comm.set_blocks(nb)
                stats[6 + i * G + j] = _time_ms(lambda: _xgmi_op(comm, op, a, ap, ag))
            stats[3 + i] = _time_ms(lambda: _rccl_op(op, g, a, ap, ag))
        comm.check()
    dist.all_reduce(stats, op=dist.ReduceOp.MAX, group=g)
    use, info = {}, dict(bytes=n * x.element_size())
    for i, op in enumerate(_OPS):
        bad, t_r = stats[i].item() > 0, stats[3 + i].item()
        times = stats[6 + i * G: 6 + (i + 1) * G].tolist()
        best = min(j for j, tt in enumerate(times) if tt <= 1.1 * min(times)) if timed and not bad \
            else _GRIDS.index(32)
        t_x = times[best]
        comm.op_blocks[op] = _GRIDS[best]
        if m == "xgmi" and bad:
            raise RuntimeError(f"xGMI {op} failed validation (max err {errs[i]:.3g}, timeout flag {comm.error()})")
        use[op] = not bad and (m == "xgmi" or t_x < 0.97 * t_r)
        info[op] = dict(transport="xgmi" if use[op] else "rccl", xgmi_ms=round(t_x, 3), rccl_ms=round(t_r, 3),
                        xgmi_blocks=_GRIDS[best], valid=not bad)
    info["transport"] = "/".join(f"{op}:{'xgmi' if use[op] else 'rccl'}" for op in _OPS)
    _info[id(g)] = info
    if p.global_rank == 0 and os.environ.get("DPFS_QUIET", "0") != "1":
        print(f"[dpfs] TP collectives: {info}", file=sys.stderr, flush=True)
    return _Choice(comm, use) if any(use.values()) else None


def _comm(t: torch.Tensor, p, op: str):
    if t.dtype not in (torch.bfloat16, torch.float32) or not t.is_cuda:
        return None
    key = id(p.tp_group)
    if key not in _decisions:
        _decisions[key] = _decide(t, p)
    ch = _decisions[key]
    return ch.comm if ch is not None and ch.use[op] else None


def info() -> Optional[dict]:
    p = pm.pgm
    return None if p is None else _info.get(id(p.tp_group))


def all_reduce(t: torch.Tensor, async_op: bool = True):
    """SUM over the TP group, in place.  Returns a work handle (``wait()``) or None."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        return None
    c = _comm(t, p, "all_reduce")
    if c is None:
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=p.tp_group, async_op=async_op)
    return c.all_reduce(t, async_op=async_op)


def reduce_scatter(out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
    """out = rank-th of tp_size equal row blocks of SUM(inp) over the TP group."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        out.copy_(inp.view_as(out))
        return None
    c = _comm(inp, p, "reduce_scatter")
    if c is None or inp.numel() * inp.element_size() > c.cap or inp.numel() % (8 * p.tp_size):
        return dist.reduce_scatter_tensor(out, inp, group=p.tp_group, async_op=async_op)
    return c.reduce_scatter(out, inp, async_op=async_op)


def all_gather(out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
    """out = concatenation (rank order, dim 0) of inp over the TP group."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        out.copy_(inp.view_as(out))
        return None
    c = _comm(inp, p, "all_gather")
    if c is None or inp.numel() * inp.element_size() > c.cap or inp.numel() % 8:
        return dist.all_gather_into_tensor(out, inp, group=p.tp_group, async_op=async_op)
    return c.all_gather(out, inp, async_op=async_op)


def staging(slot: int, shape, dtype: torch.dtype, op: str = "all_reduce") -> Optional[torch.Tensor]:
    """Output buffer for a GEMM whose result feeds the next TP all-reduce / reduce-scatter:
    a view of the xGMI communicator's staging slot ``slot`` (then the collective skips its
    copy-in), or None when ``op`` runs on RCCL, the group has not chosen yet, or it does not fit.
    Use one slot per in-flight chunk; a slot may be rewritten once the collective that read
    it has been waited."""
    p = pm.pgm
    if p is None or p.tp_size == 1 or os.environ.get("DPFS_XGMI_STAGING", "1") == "0":
        return None
    ch = _decisions.get(id(p.tp_group))
    if ch is None or not ch.use[op]:
        return None
    return ch.comm.staging(slot, shape, dtype)


def check():
    """Raise if any xGMI call of this process timed out (cheap: one host-mapped word)."""
    p = pm.pgm
    if p is None:
        return
    ch = _decisions.get(id(p.tp_group))
    if ch is not None:
        ch.comm.check()
