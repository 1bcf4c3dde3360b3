"""Transport of the tensor-parallel collectives: RCCL (two ways) or xGMI peer memory.

``DPFS_TP_COMM`` = ``auto`` (default) | ``rccl`` | ``native`` | ``xgmi`` | ``relay``.

* ``rccl``: ``torch.distributed`` on the TP group (ProcessGroupNCCL; ``nccl`` = RCCL on ROCm).
* ``native``: :class:`~.rccl.RcclComm`, the RCCL C API on our own side stream.
* ``xgmi``: :class:`~.xgmi.XgmiComm` (hand-written peer-memory kernels, all links at once).
* ``relay``: :class:`~.relay.RelayComm` (TP = 2 with other pairs on the node: each pair's
  exchange split over the direct link and two-hop paths through every other GPU, RCCL
  point-to-point on the WORLD group).  Every rank of the WORLD takes part in each relayed
  collective, so when it is a candidate the validation / timing results are reduced over the
  WORLD and every TP group reaches the same decision.
* ``auto``: on the first TP collective of the process, every TP rank builds the xGMI
  communicator and, for each of all-reduce, reduce-scatter and all-gather separately, checks
  its results against an fp32 ProcessGroupNCCL sum on a rank-dependent tensor of the live
  message size and times both (xGMI at several grid widths).  An op leaves ProcessGroupNCCL
  only if xGMI was correct on every rank and at least 3 % faster (max over ranks).  Every
  rank reaches the same decisions (they are computed from all-reduced numbers), so the call
  sequence stays identical across the group.  (``native`` runs the same RCCL kernels as
  ProcessGroupNCCL, so ``auto`` does not open a second RCCL communicator: two communicators
  with kernels in flight at once are only safe while the GPU can hold both.)

Only the TP group's activation / activation-gradient collectives go through here; DP gradient
buckets, the CE statistics gather and init broadcasts stay on ProcessGroupNCCL.

Rehearsal hook: ``DPFS_TP_COMM_AUTO_ANY_BACKEND=1`` lets ``auto`` run its whole decision
(validation, timing, grid choice, WORLD reductions, relay candidate) on a non-``nccl`` backend,
i.e. gloo with several ranks on one GPU (xGMI + relay candidates) or on the CPU (relay
candidate only).  The "rccl" column is then the gloo process group.  Tests use it to pin that
every rank reaches the same decisions before the first real multi-GPU run.
"""
from __future__ import annotations

import os
import sys
import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

from . import process_manager as pm

_OPS = ("all_reduce", "reduce_scatter", "all_gather")
_GRIDS = (8, 16, 32, 64)
_decisions: Dict[int, Optional["_Choice"]] = {}   # id(tp_group) -> per-op transport (None = RCCL)
_info: Dict[int, dict] = {}


def mode() -> str:
    m = os.environ.get("DPFS_TP_COMM", "auto")
    assert m in ("auto", "rccl", "native", "xgmi", "relay"), \
        f"DPFS_TP_COMM={m!r}: expected auto | rccl | native | xgmi | relay"
    return m


def _auto_any_backend() -> bool:
    return os.environ.get("DPFS_TP_COMM_AUTO_ANY_BACKEND", "0") == "1"


def _sync(dev_is_cuda: bool):
    if dev_is_cuda:
        torch.cuda.synchronize()


def _time_ms(fn, cuda: bool = True, reps: int = 5) -> float:
    fn()
    _sync(cuda)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    _sync(cuda)
    return 1000 * (time.perf_counter() - t0) / reps


class _Choice:
    """The group's communicators and which transport each op uses ("rccl" = ProcessGroupNCCL)."""

    def __init__(self, xgmi, native, use: Dict[str, str]):
        self.xgmi, self.native, self.use = xgmi, native, use

    relay = None

    def comm(self, op: str):
        u = self.use[op]
        return {"xgmi": self.xgmi, "native": self.native, "relay": self.relay}.get(u)


def _run_op(comm, op: str, x, part, gathered, timeout_s=None):
    """One blocking collective on ``comm`` (XgmiComm / RcclComm) or, for comm = (None, group),
    on ProcessGroupNCCL."""
    if isinstance(comm, tuple):
        g = comm[1]
        if op == "all_reduce":
            dist.all_reduce(x, group=g)
        elif op == "reduce_scatter":
            _pg_reduce_scatter(part, x, g)
        else:
            _pg_all_gather(gathered, part, g)
        return
    kw = {} if timeout_s is None else {"timeout_s": timeout_s}
    if op == "all_reduce":
        comm.all_reduce(x, async_op=False, **kw)
    elif op == "reduce_scatter":
        comm.reduce_scatter(part, x, async_op=False, **kw)
    else:
        comm.all_gather(gathered, part, async_op=False, **kw)


def _gloo_cuda(t: torch.Tensor, g) -> bool:
    return t.is_cuda and dist.get_backend(g) == "gloo"


def _pg_reduce_scatter(out: torch.Tensor, inp: torch.Tensor, g, async_op: bool = False):
    """``dist.reduce_scatter_tensor`` on the process group; gloo with device tensors (the
    one-GPU multi-rank rehearsal) goes through an all-reduce of a copy instead."""
    if _gloo_cuda(inp, g):
        tmp = inp.contiguous().clone()
        dist.all_reduce(tmp, group=g)
        out.view(-1).copy_(tmp.view(dist.get_world_size(g), -1)[dist.get_rank(g)])
        return None
    return dist.reduce_scatter_tensor(out, inp, group=g, async_op=async_op)


def _pg_all_gather(out: torch.Tensor, inp: torch.Tensor, g, async_op: bool = False):
    if _gloo_cuda(inp, g):
        W, r = dist.get_world_size(g), dist.get_rank(g)
        pad = torch.zeros(W, inp.numel(), dtype=inp.dtype, device=inp.device)
        pad[r].copy_(inp.reshape(-1))
        dist.all_reduce(pad, group=g)
        out.view(-1).copy_(pad.view(-1))
        return None
    return dist.all_gather_into_tensor(out, inp, group=g, async_op=async_op)


def _build(kind: str, g, forced: bool):
    """Communicator of ``kind`` on every rank of g, or None on every rank if any rank failed."""
    ok = torch.ones(1, device="cuda" if torch.cuda.is_available() else "cpu")
    comm, why = None, ""
    try:
        if kind == "xgmi":
            from .xgmi import XgmiComm
            comm = XgmiComm(g)
        else:
            from .rccl import RcclComm
            comm = RcclComm(g)
    except Exception as e:   # IPC / RCCL unavailable: the whole group does without it
        ok.zero_()
        why = f"setup failed: {e}"
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=g)
    if ok.item() == 0:
        if forced:
            raise RuntimeError(f"DPFS_TP_COMM={kind} but the communicator could not be built ({why})")
        return None
    return comm


_fixed_shapes = False


def set_fixed_shapes(v: bool = True):
    """Declare that every rank of the WORLD passes the same message sizes to every TP
    collective (synthetic data / fixed-length batches: bench.py, ``train.py --synthetic``).
    Only then does ``auto`` consider the relayed transport, whose exchanges pair every rank
    with every other (parallel/relay.py pads to a WORLD-agreed size otherwise)."""
    global _fixed_shapes
    _fixed_shapes = bool(v)


def _relay_possible(p) -> bool:
    W = dist.get_world_size()
    return p.tp_size == 2 and W >= 4 and W % 2 == 0


def _decide(t: torch.Tensor, p) -> Optional[_Choice]:
    m = mode()
    backend = dist.get_backend(p.tp_group)
    any_be = m == "auto" and _auto_any_backend()
    if m == "rccl" or (m == "auto" and backend != "nccl" and not any_be):
        return None
    if not t.is_cuda and not (m == "relay" or any_be):
        return None
    g = p.tp_group
    W, r = p.tp_size, p.tp_rank
    kinds = [m] if m != "auto" else (["xgmi"] if t.is_cuda else [])
    relay_cand = (m == "relay" or (m == "auto" and _fixed_shapes)) and _relay_possible(p)
    if m == "relay" and not _relay_possible(p):
        raise RuntimeError("DPFS_TP_COMM=relay needs TP = 2 and at least two TP pairs")
    comms = {k: _build(k, g, forced=m != "auto") for k in kinds if k != "relay"}
    comms = {k: c for k, c in comms.items() if c is not None}
    if relay_cand:
        # every decision input below is reduced over the WORLD, so every pair must hold the
        # same candidate set: drop xGMI everywhere unless every pair built it
        have = torch.tensor([1.0 if "xgmi" in comms else 0.0], device=t.device if t.is_cuda and backend == "nccl" else "cpu")
        dist.all_reduce(have, op=dist.ReduceOp.MIN)
        if have.item() == 0.0:
            comms.pop("xgmi", None)
        from .relay import RelayComm
        comms["relay"] = RelayComm(p)
        comms["relay"].fixed_shapes = _fixed_shapes
    # relayed ops involve every rank of the WORLD: reduce every decision input over it
    red_group = None if relay_cand else g
    if not comms:
        return None
    # Correctness of every op on a rank-dependent tensor of the live size, against fp32 sums
    # (ProcessGroup all-reduce only: the all-gather oracle is a zero-padded sum, exact).
    n = t.numel()
    if "xgmi" in comms:
        n = min(n, comms["xgmi"]._max_elems(t))
    n = max(8 * W, n - n % (8 * W))
    if relay_cand:   # relayed exchanges pair every rank with every other: one size for the WORLD
        nt = torch.tensor([n], dtype=torch.int64, device=t.device if backend == "nccl" else "cpu")
        dist.all_reduce(nt, op=dist.ReduceOp.MIN)
        n = int(nt.item())
    gen = torch.Generator(device=t.device).manual_seed(4321 + r)
    x = torch.randn(n, generator=gen, device=t.device).to(t.dtype)
    ref = x.float().clone()      # (an fp32 x must not be summed in place: it is the test input)
    dist.all_reduce(ref, group=g)
    mine = x.view(W, -1)[r]
    pad = torch.zeros(W, n // W, device=t.device)
    pad[r] = mine.float()
    dist.all_reduce(pad, group=g)
    tol = 1e-2 * max(1.0, ref.abs().max().item())
    kl = sorted(comms)
    bad = torch.zeros(len(kl), 3, device=t.device)
    errs = {}
    for a, k in enumerate(kl):
        c = comms[k]
        y, part, gathered = x.clone(), torch.empty_like(mine), torch.empty_like(x)
        to = 30.0 if k == "xgmi" else None
        _run_op(c, "all_reduce", y, None, None, to)
        _run_op(c, "reduce_scatter", x, part, None, to)
        _run_op(c, "all_gather", None, mine, gathered, to)
        _sync(t.is_cuda)
        e = [(y.float() - ref).abs().max().item(), (part.float() - ref.view(W, -1)[r]).abs().max().item(),
             (gathered.float() - pad.view(-1)).abs().max().item()]
        timed_out = k == "xgmi" and c.error() != 0
        errs[k] = e
        for i in range(3):
            good = not timed_out and (e[i] <= tol if i < 2 else e[i] == 0.0)
            bad[a, i] = 0.0 if good else 1.0
    dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=red_group)
    if m != "auto" and bad.sum().item() > 0:
        raise RuntimeError(f"DPFS_TP_COMM={m}: collectives failed validation (max errors {errs[m]})")
    # Timing (ProcessGroupNCCL backend only).  xGMI workgroups per call (1024 threads each):
    # every CU that holds one cannot also hold a 2-wave-per-SIMD GEMM block, so per op take
    # the narrowest grid within 10 % of the fastest one measured in isolation.
    G = len(_GRIDS)
    cols = ["rccl"] + [k for k in kl if k != "xgmi"] + ([f"xgmi/{nb}" for nb in _GRIDS] if "xgmi" in comms else [])
    times = torch.zeros(3, len(cols), device=t.device)
    timed = m == "auto" and (backend == "nccl" or any_be)
    if timed:
        a_, ap, ag = t.detach().reshape(-1)[:n].clone(), torch.empty_like(mine), torch.empty_like(x)
        for i, op in enumerate(_OPS):
            for j, col in enumerate(cols):
                kind = col.split("/")[0]
                if kind != "rccl" and bad[kl.index(kind), i] > 0:
                    continue
                if col == "rccl":
                    c = (None, g)
                else:
                    c = comms[kind]
                    if kind == "xgmi":
                        c.set_blocks(int(col.split("/")[1]))
                times[i, j] = _time_ms(lambda c=c, op=op: _run_op(c, op, a_, ap, ag), t.is_cuda)
        if "xgmi" in comms:
            comms["xgmi"].check()
    dist.all_reduce(times, op=dist.ReduceOp.MAX, group=red_group)
    use, info = {}, dict(bytes=n * x.element_size())
    for i, op in enumerate(_OPS):
        row = times[i].tolist()
        ok = {k: bad[a, i].item() == 0 for a, k in enumerate(kl)}
        cand = {"rccl": row[0]}
        for k in ("native", "relay"):
            if k in comms and ok[k]:
                cand[k] = row[cols.index(k)]
        if "xgmi" in comms:
            xt = row[len(cols) - G:]
            jx = min(j for j, tt in enumerate(xt) if tt <= 1.1 * min(xt)) if timed else _GRIDS.index(32)
            comms["xgmi"].op_blocks[op] = _GRIDS[jx]
            if ok["xgmi"]:
                cand["xgmi"] = xt[jx]
        if m != "auto":
            choice = m
        else:
            fastest = min(cand, key=cand.get)
            choice = fastest if fastest != "rccl" and cand[fastest] < 0.97 * cand["rccl"] else "rccl"
        use[op] = choice
        info[op] = dict(transport=choice, **{f"{k}_ms": round(v, 3) for k, v in cand.items()})
        if "xgmi" in comms:
            info[op]["xgmi_blocks"] = comms["xgmi"].op_blocks[op]
    info["transport"] = "/".join(f"{op}:{use[op]}" for op in _OPS)
    _info[id(g)] = info
    if p.global_rank == 0 and os.environ.get("DPFS_QUIET", "0") != "1":
        print(f"[dpfs] TP collectives: {info}", file=sys.stderr, flush=True)
    if all(u == "rccl" for u in use.values()):
        if "xgmi" in comms:      # same decision on every rank of g: release the IPC buffers
            comms["xgmi"].close()
        return None
    ch = _Choice(comms.get("xgmi"), comms.get("native"), use)
    ch.relay = comms.get("relay")
    return ch


def _comm(t: torch.Tensor, p, op: str):
    if t.dtype not in (torch.bfloat16, torch.float32):
        return None
    if not t.is_cuda and not (mode() == "relay" or (mode() == "auto" and _auto_any_backend())):
        return None
    key = id(p.tp_group)
    if key not in _decisions:
        _decisions[key] = _decide(t, p)
    ch = _decisions[key]
    return None if ch is None else ch.comm(op)


def decision() -> Optional[dict]:
    """This rank's transport per op and the xGMI grid per op (None before the first TP
    collective or off TP): what every rank of a group must agree on."""
    p = pm.pgm
    if p is None or id(p.tp_group) not in _decisions:
        return None
    inf = _info.get(id(p.tp_group))
    if inf is None:              # no candidate transport was built: the process group
        return {"use": {op: "rccl" for op in _OPS}, "op_blocks": None}
    blocks = {op: inf[op].get("xgmi_blocks") for op in _OPS}
    return {"use": {op: inf[op]["transport"] for op in _OPS},
            "op_blocks": blocks if any(v is not None for v in blocks.values()) else None}


def reset():
    """Release every communicator built by the decisions (xGMI IPC buffers, the native RCCL
    communicator) and forget them, e.g. between two layouts measured in one process.
    Collective over each TP group that has decided (every rank must call it)."""
    for key, ch in list(_decisions.items()):
        if ch is not None:
            if ch.xgmi is not None:
                ch.xgmi.close()
            if ch.native is not None and hasattr(ch.native, "close"):
                ch.native.close()
        _decisions.pop(key, None)
        _info.pop(key, None)


def info() -> Optional[dict]:
    p = pm.pgm
    return None if p is None else _info.get(id(p.tp_group))


def _fits(c, t: torch.Tensor, mult: int) -> bool:
    """xGMI takes messages up to its buffer capacity, in 16-byte vectors; RCCL takes any."""
    if not hasattr(c, "cap"):
        return True
    return t.numel() * t.element_size() <= c.cap and t.numel() % mult == 0


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
    if c is None or not _fits(c, inp, 8 * p.tp_size):
        return _pg_reduce_scatter(out, inp, p.tp_group, async_op)
    return c.reduce_scatter(out, inp, async_op=async_op)


def all_gather(out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
    """out = concatenation (rank order, dim 0) of inp over the TP group."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        out.copy_(inp.view_as(out))
        return None
    c = _comm(inp, p, "all_gather")
    if c is None or not _fits(c, inp, 8):
        return _pg_all_gather(out, inp, p.tp_group, async_op)
    return c.all_gather(out, inp, async_op=async_op)


def staging(slot: int, shape, dtype: torch.dtype, op: str = "all_reduce") -> Optional[torch.Tensor]:
    """Output buffer for a GEMM whose result feeds the next TP all-reduce / reduce-scatter:
    a view of the xGMI communicator's staging slot ``slot`` (then the collective skips its
    copy-in), or None when ``op`` does not run on xGMI, the group has not chosen yet, or it
    does not fit.  Use one slot per in-flight chunk; a slot may be rewritten once the
    collective that read it has been waited."""
    p = pm.pgm
    if p is None or p.tp_size == 1 or os.environ.get("DPFS_XGMI_STAGING", "1") == "0":
        return None
    ch = _decisions.get(id(p.tp_group))
    if ch is None or ch.use[op] != "xgmi":
        return None
    return ch.xgmi.staging(slot, shape, dtype)


def check():
    """Raise if any xGMI call of this process timed out (one host-mapped word) or the native
    RCCL communicator reported an asynchronous error."""
    p = pm.pgm
    if p is None:
        return
    ch = _decisions.get(id(p.tp_group))
    if ch is not None:
        if ch.xgmi is not None:
            ch.xgmi.check()
        if ch.native is not None:
            ch.native.check()
