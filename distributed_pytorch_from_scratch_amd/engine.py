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
"""
from __future__ import annotations

from typing import Optional

import torch

from .models.transformer import Transformer
from .parallel import process_manager as pm
from .parallel.grad_sync import DataParallelGradSync, allreduce_sequence_parallel_grads


class TrainStep:
    def __init__(self, model: Transformer, optimizer: torch.optim.Optimizer, scheduler=None,
                 dp_bucket_mb: float = 32.0):
        self.model = model
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.sp = model.args.sequence_parallel
        p = pm.pgm
        self.dp = DataParallelGradSync(model, dp_bucket_mb) if (p is not None and p.dp_size > 1) else None

    def __call__(self, input_ids: torch.Tensor, position_ids: torch.Tensor,
                 target_ids: torch.Tensor) -> torch.Tensor:
        loss = self.model.loss(input_ids, position_ids, target_ids)
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        if self.sp:
            allreduce_sequence_parallel_grads(self.model)
        if self.dp is not None:
            self.dp.finish()
        self.optimizer.step()
        if self.scheduler is not None:
            self.scheduler.step()
        return loss.detach()
