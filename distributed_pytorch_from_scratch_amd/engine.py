"""One training step, shared by ``train.py`` and ``bench.py``.

Reference hot loop: ``train.py:94-111`` (autocast forward, gathered-logit CE, ``zero_grad``,
``backward``, ``Adam.step``, ``OneCycleLR.step``, ``loss.item()`` every step).  Here:

* forward + vocab-parallel CE (no logits all-gather), bf16 activations, fp32 master weights;
* backward with the TP all-reduces overlapped inside the linear Functions;
* sequence-parallel replicated-param grads all-reduced over TP (when SP is on), DP grads
  all-reduced in overlapped buckets (when DP > 1);
* fused Adam (one kernel) + scheduler step;
* no host synchronisation: the loss stays a device tensor; callers read it only when they
  log (the reference syncs with ``loss.item()`` on every step, ``train.py:110``).

Observability: ``timings()`` returns the last step's fwd / bwd / optimizer
milliseconds from HIP events (recorded every step, read only when asked); ``DPFS_ROCTX=1``
wraps the phases in roctx ranges for rocprofv3; ``DPFS_COMM_CHECK=1`` compares the
collective sequence of every rank after each step (``utils/comm_check.py``).
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Dict, Optional

import torch

from .models.transformer import Transformer
from .parallel import process_manager as pm
from .parallel.grad_sync import DataParallelGradSync, allreduce_sequence_parallel_grads, setup_dp_buckets
from .utils import comm_check


@contextmanager
def roctx(name: str):
    """roctx range (torch.cuda.nvtx maps to roctx on ROCm) when DPFS_ROCTX=1."""
    on = os.environ.get("DPFS_ROCTX") == "1" and torch.cuda.is_available()
    if on:
        torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        if on:
            torch.cuda.nvtx.range_pop()


class TrainStep:
    def __init__(self, model: Transformer, optimizer: torch.optim.Optimizer, scheduler=None,
                 dp_bucket_mb: float = 32.0):
        self.model = model
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.sp = model.args.sequence_parallel
        p = pm.pgm
        # The fused engine averages DP gradients itself, overlapped with its backward.
        use_hooks = p is not None and p.dp_size > 1 and not model.fused_supported()
        self.dp = DataParallelGradSync(model, dp_bucket_mb) if use_hooks else None
        if p is not None and p.dp_size > 1 and model.fused_supported():
            # the fused engines' DP bucket size: measured once here, outside the backward, and
            # MAX-reduced over every rank so all DP groups use one size
            setup_dp_buckets(next(model.parameters()).device)
        self.checker = comm_check.from_env()
        self.steps = 0
        self._ev = None

    def _event(self):
        if not torch.cuda.is_available() or not next(self.model.parameters()).is_cuda:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def __call__(self, input_ids: torch.Tensor, position_ids: torch.Tensor,
                 target_ids: torch.Tensor) -> torch.Tensor:
        e0 = self._event()
        with roctx("fwd"):
            loss = self.model.loss(input_ids, position_ids, target_ids, unit_grad=True)
        e1 = self._event()
        self.optimizer.zero_grad(set_to_none=True)
        with roctx("bwd"):
            # a cached unit gradient (autograd would fill a fresh ones tensor every step)
            g1 = getattr(self, "_unit", None)
            if g1 is None or g1.device != loss.device or g1.dtype != loss.dtype or g1.shape != loss.shape:
                g1 = self._unit = torch.ones_like(loss)
            loss.backward(g1)
            # DP first: finish() copies the DP-averaged buckets (packed during backward, before
            # any TP sum) back into .grad; the SP sum over TP must act on those copied-back grads.
            # The two sums commute, so this order gives sum_tp(mean_dp(g)).
            if self.dp is not None:
                self.dp.finish()
            if self.sp:
                allreduce_sequence_parallel_grads(self.model)
        e2 = self._event()
        with roctx("opt"):
            self.optimizer.step()
            if self.scheduler is not None:
                self.scheduler.step()
        e3 = self._event()
        self._ev = (e0, e1, e2, e3) if e0 is not None else None
        self.steps += 1
        if self.checker is not None:
            self.checker.check(f"step{self.steps}")
        return loss.detach()

    def timings(self) -> Dict[str, float]:
        """fwd / bwd / opt milliseconds of the last step (synchronises on its last event)."""
        if self._ev is None:
            return {}
        e0, e1, e2, e3 = self._ev
        e3.synchronize()
        return {"fwd_ms": e0.elapsed_time(e1), "bwd_ms": e1.elapsed_time(e2), "opt_ms": e2.elapsed_time(e3)}
