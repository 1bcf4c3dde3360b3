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
  message size, then times the candidates per op AND per size class (``SIZE_CLASSES``: small
  messages <= 1 MiB, medium <= 16 MiB, large; one representative size each): ProcessGroupNCCL,
  the xGMI two-shot kernels at several grid widths, the xGMI one-shot all-reduce (one barrier;
  small / medium classes) and the relay.  An (op, class) leaves ProcessGroupNCCL only if the
  candidate was correct on every rank and at least 3 % faster (max over ranks).  Every rank
  reaches the same decisions (they are computed from all-reduced numbers), so the call
  sequence stays identical across the group.  (``native`` runs the same RCCL kernels as
  ProcessGroupNCCL and is not an ``auto`` candidate: a second RCCL communicator whose kernels
  run while ProcessGroupNCCL's (DP buckets, CE statistics) are in flight can deadlock when the
  GPU cannot hold both at once, and RCCL refuses two ranks on one device, so it cannot be
  timed on a one-GPU rehearsal either; it stays an explicit opt-in.)

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
# (class, upper bound in bytes, representative size timed for it)
SIZE_CLASSES = (("s", 1 << 20, 512 << 10), ("m", 16 << 20, 8 << 20), ("l", None, 32 << 20))


def size_class(nbytes: int) -> str:
    for name, hi, _ in SIZE_CLASSES:
        if hi is None or nbytes <= hi:
            return name
    return SIZE_CLASSES[-1][0]
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
    """The group's communicators and the transport of each (op, size class): "rccl" =
    ProcessGroupNCCL, "xgmi" = the two-shot kernels, "xgmi1" = the one-shot all-reduce,
    "native", "relay"; ``blocks`` = the xGMI grid of each (op, class)."""

    def __init__(self, xgmi, native, use: Dict[tuple, str], blocks: Optional[Dict[tuple, int]] = None):
        self.xgmi, self.native, self.use = xgmi, native, use
        self.blocks = blocks or {}

    relay = None

    def route(self, op: str, nbytes: int):
        """(communicator, call kwargs) for a message of ``nbytes``, or None = ProcessGroupNCCL."""
        key = (op, size_class(nbytes))
        u = self.use[key]
        if u in ("xgmi", "xgmi1"):
            nb = self.blocks.get(key)
            if nb is not None and nb != self.xgmi._blocks:   # same call sequence on every rank
                self.xgmi.set_blocks(nb)
            return self.xgmi, ({"one_shot": True} if u == "xgmi1" else {})
        c = {"native": self.native, "relay": self.relay}.get(u)
        return None if c is None else (c, {})

    def uses(self, op: str, transport: str) -> bool:
        return any(v == transport for (o, _), v in self.use.items() if o == op)


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
    # One-shot all-reduce (xGMI): bit-identical to the two-shot form (same fp32 rank-order
    # sums), checked on a message that fits its capacity.
    one_shot = "xgmi" in comms and not bad[kl.index("xgmi"), 0]
    if one_shot:
        c = comms["xgmi"]
        n1 = max(8 * W, min(n, c.one_shot_cap // x.element_size()) // (8 * W) * (8 * W))
        y1, y2 = x[:n1].clone(), x[:n1].clone()
        _run_op(c, "all_reduce", y1, None, None, 30.0)
        c.all_reduce(y2, async_op=False, timeout_s=30.0, one_shot=True)
        _sync(t.is_cuda)
        ok1 = torch.tensor([1.0 if (torch.equal(y1, y2) and c.error() == 0) else 0.0], device=t.device)
        dist.all_reduce(ok1, op=dist.ReduceOp.MIN, group=red_group)
        one_shot = ok1.item() == 1.0
    # Timing (ProcessGroupNCCL backend only), per op and size class at one representative
    # size per class.  xGMI workgroups per call (1024 threads each): every CU that holds one
    # cannot also hold a 2-wave-per-SIMD GEMM block, so per (op, class) take the narrowest grid
    # within 10 % of the fastest one measured in isolation.
    G = len(_GRIDS)
    xg = "xgmi" in comms
    cols = ["rccl"] + [k for k in kl if k != "xgmi"] + ([f"xgmi/{nb}" for nb in _GRIDS] if xg else []) \
        + ([f"xgmi1/{nb}" for nb in _GRIDS] if one_shot else [])
    NC = len(SIZE_CLASSES)
    times = torch.full((3, NC, len(cols)), float("inf"), device=t.device)
    timed = m == "auto" and (backend == "nccl" or any_be)
    cap_el = comms["xgmi"]._max_elems(t) if xg else None
    sizes = []
    for ci, (cname, hi, rep) in enumerate(SIZE_CLASSES):
        ne = max(8 * W, rep // t.element_size())
        if cap_el is not None:
            ne = min(ne, cap_el)
        ne -= ne % (8 * W)
        sizes.append(ne)
    if relay_cand:   # one size per class for the WORLD (relayed exchanges pair every rank)
        st_ = torch.tensor(sizes, dtype=torch.int64, device=t.device if backend == "nccl" else "cpu")
        dist.all_reduce(st_, op=dist.ReduceOp.MIN)
        sizes = [int(v) for v in st_.tolist()]
    if timed:
        for ci in range(NC):
            ne = sizes[ci]
            gen2 = torch.Generator(device=t.device).manual_seed(99 + r)
            a_ = torch.randn(ne, generator=gen2, device=t.device).to(t.dtype)
            ap, ag = torch.empty(ne // W, dtype=t.dtype, device=t.device), torch.empty_like(a_)
            for i, op in enumerate(_OPS):
                for j, col in enumerate(cols):
                    kind = col.split("/")[0]
                    base = "xgmi" if kind == "xgmi1" else kind
                    if kind != "rccl" and bad[kl.index(base), i] > 0:
                        continue
                    if kind == "xgmi1" and (op != "all_reduce" or ne * t.element_size() > comms["xgmi"].one_shot_cap):
                        continue
                    if col == "rccl":
                        fn = (lambda op=op: _run_op((None, g), op, a_, ap, ag))
                    elif kind in ("xgmi", "xgmi1"):
                        c = comms["xgmi"]

                        def fn(c=c, op=op, nb=int(col.split("/")[1]), one=kind == "xgmi1"):
                            c.set_blocks(nb)
                            if one:
                                c.all_reduce(a_, async_op=False, one_shot=True)
                            else:
                                _run_op(c, op, a_, ap, ag)
                    else:
                        fn = (lambda c=comms[kind], op=op: _run_op(c, op, a_, ap, ag))
                    times[i, ci, j] = _time_ms(fn, t.is_cuda)
    # A barrier that timed out on ANY rank while timing (its flag is per rank) takes the xGMI
    # kernels out of the running on every rank alike, so the group still decides the same.
    xerr = torch.tensor([float(comms["xgmi"].error()) if xg else 0.0], device=t.device)
    dist.all_reduce(xerr, op=dist.ReduceOp.MAX, group=red_group)
    if xerr.item() > 0:
        comms["xgmi"].clear_error()
        for j, c_ in enumerate(cols):
            if c_.startswith("xgmi"):
                times[:, :, j] = float("inf")
        if p.global_rank == 0:
            print("[dpfs] TP collectives: an xGMI barrier timed out while timing; xGMI is not used",
                  file=sys.stderr, flush=True)
    dist.all_reduce(times, op=dist.ReduceOp.MAX, group=red_group)
    use, blocks, info = {}, {}, dict(bytes=n * x.element_size(),
                                     class_bytes={c[0]: sizes[i] * x.element_size() for i, c in enumerate(SIZE_CLASSES)})
    for i, op in enumerate(_OPS):
        info[op] = {}
        ok = {k: bad[a, i].item() == 0 for a, k in enumerate(kl)}
        for ci, (cname, _, _) in enumerate(SIZE_CLASSES):
            row = times[i, ci].tolist()
            cand = {"rccl": row[0]}
            for k in ("native", "relay"):
                if k in comms and ok[k]:
                    cand[k] = row[cols.index(k)]
            grid = {}
            for kind in ("xgmi", "xgmi1"):
                js = [j for j, c_ in enumerate(cols) if c_.split("/")[0] == kind]
                if not js or not ok.get("xgmi", False):
                    continue
                xt = [row[j] for j in js]
                if min(xt) == float("inf"):
                    continue
                jx = min(j for j, tt in enumerate(xt) if tt <= 1.1 * min(xt)) if timed else _GRIDS.index(32)
                grid[kind] = _GRIDS[jx]
                cand[kind] = xt[jx]
            if m == "auto":
                fastest = min(cand, key=cand.get)
                choice = fastest if fastest != "rccl" and cand[fastest] < 0.97 * cand["rccl"] else "rccl"
            else:
                choice = m if m != "xgmi" or "xgmi" in grid or not timed else m
            use[(op, cname)] = choice
            if choice in grid:
                blocks[(op, cname)] = grid[choice]
            elif choice == "xgmi":
                blocks[(op, cname)] = grid.get("xgmi", 32)
            info[op][cname] = dict(transport=choice, **{f"{k}_ms": round(v, 3) for k, v in cand.items()
                                                         if v != float("inf")})
            if (op, cname) in blocks:
                info[op][cname]["xgmi_blocks"] = blocks[(op, cname)]
    info["transport"] = "/".join(f"{op}:" + ",".join(f"{c[0]}={use[(op, c[0])]}" for c in SIZE_CLASSES)
                                 for op in _OPS)
    _info[id(g)] = info
    if p.global_rank == 0 and os.environ.get("DPFS_QUIET", "0") != "1":
        print(f"[dpfs] TP collectives: {info}", file=sys.stderr, flush=True)
    if all(u == "rccl" for u in use.values()):
        if "xgmi" in comms:      # same decision on every rank of g: release the IPC buffers
            comms["xgmi"].close()
        return None
    ch = _Choice(comms.get("xgmi"), comms.get("native"), use, blocks)
    ch.relay = comms.get("relay")
    return ch


def _comm(t: torch.Tensor, p, op: str, nbytes: Optional[int] = None):
    """(communicator, kwargs) for this op and message size, or None (ProcessGroupNCCL)."""
    if t.dtype not in (torch.bfloat16, torch.float32):
        return None
    if not t.is_cuda and not (mode() == "relay" or (mode() == "auto" and _auto_any_backend())):
        return None
    key = id(p.tp_group)
    if key not in _decisions:
        t0 = time.perf_counter()
        _decisions[key] = _decide(t, p)
        if p.global_rank == 0 and os.environ.get("DPFS_QUIET") != "1":
            tr = (_info.get(key) or {}).get("transport")
            print(f"[dpfs] TP collectives decided in {time.perf_counter() - t0:.1f} s: {tr}", file=sys.stderr,
                  flush=True)
    ch = _decisions[key]
    return None if ch is None else ch.route(op, t.numel() * t.element_size() if nbytes is None else nbytes)


def decision() -> Optional[dict]:
    """This rank's transport and xGMI grid per op and size class (None before the first TP
    collective or off TP): what every rank of a group must agree on."""
    p = pm.pgm
    if p is None or id(p.tp_group) not in _decisions:
        return None
    keys = [f"{op}/{c[0]}" for op in _OPS for c in SIZE_CLASSES]
    inf = _info.get(id(p.tp_group))
    if inf is None:              # no candidate transport was built: the process group
        return {"use": {k: "rccl" for k in keys}, "op_blocks": None}
    use = {f"{op}/{c}": inf[op][c]["transport"] for op in _OPS for c, _, _ in SIZE_CLASSES}
    blocks = {f"{op}/{c}": inf[op][c].get("xgmi_blocks") for op in _OPS for c, _, _ in SIZE_CLASSES}
    return {"use": use, "op_blocks": blocks if any(v is not None for v in blocks.values()) else None}


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
    from . import grad_sync
    grad_sync.reset()      # cached DP bucket sizes are keyed by the (replaced) process groups


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
    r = _comm(t, p, "all_reduce")
    if r is None:
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=p.tp_group, async_op=async_op)
    c, kw = r
    return c.all_reduce(t, async_op=async_op, **kw)


def reduce_scatter(out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
    """out = rank-th of tp_size equal row blocks of SUM(inp) over the TP group."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        out.copy_(inp.view_as(out))
        return None
    r = _comm(inp, p, "reduce_scatter")
    if r is None or not _fits(r[0], inp, 8 * p.tp_size):
        return _pg_reduce_scatter(out, inp, p.tp_group, async_op)
    return r[0].reduce_scatter(out, inp, async_op=async_op)


def all_gather(out: torch.Tensor, inp: torch.Tensor, async_op: bool = True):
    """out = concatenation (rank order, dim 0) of inp over the TP group."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        out.copy_(inp.view_as(out))
        return None
    r = _comm(inp, p, "all_gather", out.numel() * out.element_size())   # class of the gathered size
    if r is None or not _fits(r[0], inp, 8):
        return _pg_all_gather(out, inp, p.tp_group, async_op)
    return r[0].all_gather(out, inp, async_op=async_op)


def staging(slot: int, shape, dtype: torch.dtype, op: str = "all_reduce") -> Optional[torch.Tensor]:
    """Output buffer for a GEMM whose result feeds the next TP all-reduce / reduce-scatter:
    a view of the xGMI communicator's staging slot ``slot`` (then the collective skips its
    copy-in), or None when ``op`` does not run on xGMI, the group has not chosen yet, or it
    does not fit.  Use one slot per in-flight chunk; a slot may be rewritten once the
    collective that read it has been waited."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        return None
    ch = _decisions.get(id(p.tp_group))
    if ch is None:
        return None
    numel = 1
    for d_ in shape:
        numel *= d_
    nbytes = numel * torch.empty((), dtype=dtype).element_size()
    # staged only where this size runs on the two-shot kernels (the one-shot form reads its
    # input after barriers the staging slot's reuse does not wait for)
    if ch.use.get((op, size_class(nbytes))) != "xgmi":
        return None
    return ch.xgmi.staging(slot, shape, dtype)


def check():
    """Raise if any xGMI call of this process timed out (one host-mapped word) or the native
    RCCL communicator reported an asynchronous error.  Also raises on the kernels' own
    host-mapped error words (the stream-K GEMM hand-off, ``_ext.check_device_errors``)."""
    from ..ops import _ext
    _ext.check_device_errors()
    p = pm.pgm
    if p is None:
        return
    ch = _decisions.get(id(p.tp_group))
    if ch is not None:
        if ch.xgmi is not None:
            ch.xgmi.check()
        if ch.native is not None:
            ch.native.check()
