"""Failure detection helpers (extension; the reference relies on mp.spawn's fail-fast only).

* ``Heartbeat``: every rank publishes ``(step, wall time)`` to the c10d TCPStore; rank 0's
  background thread flags ranks whose heartbeat is older than ``stale_s`` (hung collective,
  dead GPU) and, with ``abort_on_stale``, aborts the job so the launcher tears it down instead
  of hanging until the RCCL watchdog timeout.
* ``maybe_inject_fault``: deterministic fault injection for tests (``--fault_inject_step``):
  the chosen rank raises at the given step, which must take the whole job down (fail-fast).
* RCCL's own watchdog is armed through ``init_process_group(timeout=...)`` in
  ``utils/dist.py``.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time

import torch.distributed as dist


class InjectedFault(RuntimeError):
    pass


def maybe_inject_fault(fault_step: int, step: int, rank: int, target_rank: int = None) -> None:
    if fault_step is None or fault_step < 0 or step != fault_step:
        return
    tr = int(os.environ.get("DPFS_FAULT_RANK", "0")) if target_rank is None else target_rank
    if rank == tr:
        raise InjectedFault(f"injected fault at step {step} on rank {rank}")


class Heartbeat:
    def __init__(self, interval_s: float = 30.0, stale_s: float = 600.0, abort_on_stale: bool = False,
                 max_hold_s: float = 3600.0):
        self.interval_s, self.stale_s, self.abort = interval_s, stale_s, abort_on_stale
        self.max_hold_s = max_hold_s
        self.store = None
        self._last = 0.0
        self._stop = threading.Event()
        self.stale_ranks = []
        try:
            from torch.distributed import distributed_c10d as c10d
            self.store = c10d._get_default_store()
        except Exception:
            self.store = None
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self._thread = None
        if self.store is not None and self.rank == 0 and self.world > 1:
            self._thread = threading.Thread(target=self._watch, daemon=True)
            self._thread.start()

    def beat(self, step: int, force: bool = False) -> None:
        now = time.time()
        if self.store is None or (not force and now - self._last < self.interval_s):
            return
        self._last = now
        self._step = step
        try:
            self.store.set(f"dpfs_hb/{self.rank}", f"{step}:{now}")
        except Exception:
            pass

    @contextlib.contextmanager
    def hold(self, step: int):
        """A phase that legitimately runs longer than ``stale_s`` without steps (checkpoint
        save and the barrier behind it, evaluation, an epoch-boundary loader restart): this
        rank is not judged stale inside it until ``max_hold_s`` has passed (the marker carries
        that deadline, so a rank killed inside a hold -- no exit beat -- is flagged once it
        expires), and it beats on entry and exit."""
        self.beat(step, force=True)
        if self.store is not None:
            try:
                self.store.set(f"dpfs_hb/{self.rank}", f"{step}:hold:{time.time() + self.max_hold_s}")
            except Exception:
                pass
        try:
            yield
        finally:
            self.beat(step, force=True)

    def _watch(self):
        while not self._stop.wait(self.interval_s):
            now, stale = time.time(), []
            for r in range(self.world):
                try:
                    if not self.store.check([f"dpfs_hb/{r}"]):
                        continue
                    parts = self.store.get(f"dpfs_hb/{r}").decode().split(":")
                    if len(parts) == 3 and parts[1] == "hold":   # step:hold:deadline
                        if now > float(parts[2]):
                            stale.append(r)
                        continue
                    if now - float(parts[1]) > self.stale_s:
                        stale.append(r)
                except Exception:
                    continue
            self.stale_ranks = stale
            if stale:
                print(f"[heartbeat] stale ranks (> {self.stale_s}s): {stale}", flush=True)
                if self.abort:
                    os._exit(17)

    def stop(self):
        self._stop.set()
