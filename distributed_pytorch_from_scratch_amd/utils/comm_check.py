"""Collective-sequence checker: catches rank divergence, the classic TP deadlock.

With ``DPFS_COMM_CHECK=1`` (or ``CollectiveChecker().install()``) every ``torch.distributed``
collective the framework issues is recorded as ``(op, shape, dtype, group size)`` into a
running per-rank hash. At each ``check(tag)``, for example once per training step
(``engine.TrainStep`` does this), every rank publishes its hash and its last few records
through the c10d store. It then compares them with the other ranks' and raises with both
op lists on the first mismatch. A rank that does not arrive within the timeout is reported
by number. It is probably stuck in a collective the others never issued.

The comparison goes through the TCPStore, not through a collective, so a diverged sequence
is reported instead of hanging the check itself. There is no reference counterpart
(SURVEY.md §5 "Race detection / sanitizers").
"""
from __future__ import annotations

import hashlib
import os
from collections import deque
from typing import Optional

import torch
import torch.distributed as dist

_WRAPPED = ("all_reduce", "all_gather", "all_gather_into_tensor", "reduce_scatter_tensor", "broadcast",
            "reduce_scatter", "barrier")


class CollectiveDivergence(RuntimeError):
    pass


class CollectiveChecker:
    def __init__(self, timeout_s: float = 120.0, history: int = 8):
        self.timeout_s = timeout_s
        self.h = hashlib.sha1()
        self.count = 0
        self.recent = deque(maxlen=history)
        self._orig = {}
        self._store = None

    # ---------------------------------------------------------------- recording ----
    def record(self, op: str, t: Optional[torch.Tensor], group=None) -> None:
        n = dist.get_world_size(group) if dist.is_initialized() else 1
        desc = f"{op}{tuple(t.shape) if t is not None else ()}:{str(t.dtype) if t is not None else '-'}:g{n}"
        self.h.update(desc.encode())
        self.count += 1
        self.recent.append(f"#{self.count} {desc}")

    def install(self) -> "CollectiveChecker":
        for name in _WRAPPED:
            fn = getattr(dist, name, None)
            if fn is None or name in self._orig:
                continue
            self._orig[name] = fn

            def wrapper(*args, __fn=fn, __name=name, **kw):
                t = None
                for a in args:
                    if isinstance(a, torch.Tensor):
                        t = a
                        break
                    if isinstance(a, (list, tuple)) and a and isinstance(a[0], torch.Tensor):
                        t = a[0]
                        break
                self.record(__name, t, kw.get("group"))
                return __fn(*args, **kw)
            setattr(dist, name, wrapper)
        return self

    def uninstall(self) -> None:
        for name, fn in self._orig.items():
            setattr(dist, name, fn)
        self._orig.clear()

    # ------------------------------------------------------------------ checking ----
    def _get_store(self):
        if self._store is None:
            from torch.distributed import distributed_c10d as c10d
            self._store = c10d._get_default_store()
        return self._store

    def check(self, tag) -> None:
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return
        store = self._get_store()
        rank, world = dist.get_rank(), dist.get_world_size()
        mine = f"{self.count}:{self.h.hexdigest()}"
        store.set(f"dpfs_cc/{tag}/{rank}", mine + "|" + " ; ".join(self.recent))
        keys = [f"dpfs_cc/{tag}/{r}" for r in range(world)]
        import datetime
        try:
            store.wait(keys, datetime.timedelta(seconds=self.timeout_s))
        except Exception as e:  # a rank never reached this check point
            missing = [r for r, k in enumerate(keys) if not store.check([k])]
            raise CollectiveDivergence(f"[rank {rank}] ranks {missing} did not reach collective check '{tag}' "
                                       f"within {self.timeout_s}s (last ops here: {list(self.recent)})") from e
        for r, k in enumerate(keys):
            other = store.get(k).decode()
            if other.split("|")[0] != mine:
                raise CollectiveDivergence(
                    f"collective sequence diverged at check '{tag}': rank {rank} issued {self.count} ops "
                    f"[{' ; '.join(self.recent)}] but rank {r} reports {other}")


_GLOBAL: Optional[CollectiveChecker] = None


def from_env() -> Optional[CollectiveChecker]:
    """The process-wide checker if ``DPFS_COMM_CHECK=1`` (installed on first use)."""
    global _GLOBAL
    if os.environ.get("DPFS_COMM_CHECK", "0") not in ("1", "true", "yes"):
        return None
    if _GLOBAL is None:
        _GLOBAL = CollectiveChecker().install()
    return _GLOBAL
