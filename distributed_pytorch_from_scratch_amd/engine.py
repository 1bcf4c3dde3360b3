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


class GraphTrainStep:
    """A :class:`TrainStep` whose forward + backward replay from one HIP graph.

    The step is ~300 kernel launches (GEMMs with fused epilogues, attention, norms, CE,
    embedding sort on a side stream); eagerly the host issues them one by one, and wherever the
    host falls behind the GPU idles between kernels.  After the eager warmup steps (per-shape
    GEMM selection, workspaces, the Adam descriptor table) the first call captures the forward
    and backward into a graph (``torch.cuda.graph``: the activations live in the graph's private
    pool at fixed addresses, the gradients stay where the eager steps put them); every call then
    copies the batch into the captured input buffers, replays the graph and runs the fused Adam
    (one kernel, eagerly: its learning rate / bias corrections change per step).

    Single-process steps only (no DP / TP group: their collectives and bucket hooks stay eager).
    The work per step is identical to :class:`TrainStep`'s -- only the launch path changes.
    """

    def __init__(self, step: TrainStep):
        p = pm.pgm
        assert p is None or (p.dp_size == 1 and p.tp_size == 1), "GraphTrainStep: single-rank steps only"
        self.step = step
        self.graph = None
        self.loss = None
        self.steps = 0

    def _capture(self, input_ids, position_ids, target_ids):
        st = self.step
        self.ids, self.pos, self.tgt = input_ids.clone(), position_ids.clone(), target_ids.clone()
        self.unit = torch.ones((), device=input_ids.device, dtype=torch.float32)
        torch.cuda.synchronize()
        # no .grad before the capture: the engine's backward assigns its gradient-arena views as
        # the parameters' .grad (a host-side assignment that outlives the capture) and writes,
        # rather than accumulates, them -- every replay refreshes the same tensors in place
        st.optimizer.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = st.model.loss(self.ids, self.pos, self.tgt, unit_grad=True)
            loss.backward(self.unit.to(loss.dtype).expand_as(loss))
        torch.cuda.synchronize()
        self.graph, self.loss = g, loss.detach()

    def __call__(self, input_ids: torch.Tensor, position_ids: torch.Tensor,
                 target_ids: torch.Tensor) -> torch.Tensor:
        st = self.step
        if self.graph is None:
            self._capture(input_ids, position_ids, target_ids)
        if input_ids.data_ptr() != self.ids.data_ptr():
            self.ids.copy_(input_ids, non_blocking=True)
            self.tgt.copy_(target_ids, non_blocking=True)
            if position_ids.data_ptr() != self.pos.data_ptr():
                self.pos.copy_(position_ids, non_blocking=True)
        self.graph.replay()
        st.optimizer.step()
        if st.scheduler is not None:
            st.scheduler.step()
        self.steps += 1
        return self.loss
