"""Fused multi-tensor Adam.

Drop-in for ``torch.optim.Adam`` (reference ``train.py:83``): same hyper-parameters,
``param_groups`` (so ``OneCycleLR`` with momentum cycling works), ``state_dict()`` with the
same per-parameter ``step``/``exp_avg``/``exp_avg_sq`` entries.

On the GPU one ``adam_k`` launch (``csrc/kernels/adam.hip``) updates every parameter of a
group and refreshes the bf16 compute shadows the GEMMs read (``ops.dispatch.shadow``), so
there is no per-step cast kernel.  The device descriptor table is built once (rebuilt only if a
parameter or shadow moves); fresh gradient tensors are patched in by a one-block kernel whose
pointers travel as kernel arguments, so a step never waits on a host -> device copy.
On CPU the same math runs through ``ops.reference.adam_step``.

Optional ``max_grad_norm`` clips by the global L2 norm (sum over TP-sharded params across the
TP group, replicated params counted once) without a host synchronisation: the clip
coefficient stays on the device and scales the gradients inside the Adam kernel.
"""
from __future__ import annotations

import math
from typing import Iterable, Optional

import torch
import torch.distributed as dist

from . import _ext, reference


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: Optional[float] = None,
                 norm_group=None, replicated_params=None):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.max_grad_norm = max_grad_norm
        self.norm_group = norm_group
        self._replicated = set(id(p) for p in (replicated_params or []))
        self._tables = {}

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._tables = {}   # the cached device tables point at the replaced moment buffers

    def _shadow_for(self, p):
        from .dispatch import peek_shadow
        s = peek_shadow(p)
        if s is None or s.dtype != torch.bfloat16:
            s = p.detach().to(torch.bfloat16)
            p._dpfs_shadow = (p._version, s)
        return s

    @torch.no_grad()
    def _clip_coef(self, params):
        """Device scalar min(1, max_norm / (||g|| + 1e-6))."""
        dev = params[0].device
        sq_local = torch.zeros((), device=dev, dtype=torch.float32)
        sq_rep = torch.zeros((), device=dev, dtype=torch.float32)
        for p in params:
            s = p.grad.float().pow(2).sum()
            if id(p) in self._replicated:
                sq_rep += s
            else:
                sq_local += s
        if self.norm_group is not None and dist.is_initialized() and dist.get_world_size(self.norm_group) > 1:
            dist.all_reduce(sq_local, group=self.norm_group)
        norm = torch.sqrt(sq_local + sq_rep)
        self.last_grad_norm = norm
        return torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0).reshape(1)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            lr = group["lr"]
            b1, b2 = group["betas"]
            eps, wd = group["eps"], group["weight_decay"]
            for p in params:
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
            step = int(self.state[params[0]]["step"].item())
            coef = self._clip_coef(params) if self.max_grad_norm else None
            if params[0].is_cuda:
                C = _ext.require()
                from .dispatch import peek_shadow
                # 2-D weights always carry a bf16 compute shadow; 1-D params only when a GEMM
                # epilogue reads one (a hipBLASLt bias, ops.gemm_select).
                shadows = [self._shadow_for(p) if (p.dim() >= 2 or peek_shadow(p) is not None) else None
                           for p in params]
                # Every pointer the device table holds is part of the key: load_state_dict()
                # swaps in new moment tensors, which must force a rebuild.
                key = tuple((p.data_ptr(), s.data_ptr() if s is not None else 0, p.numel(),
                             self.state[p]["exp_avg"].data_ptr(), self.state[p]["exp_avg_sq"].data_ptr())
                            for p, s in zip(params, shadows))
                grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in params]
                gkey = tuple(g.data_ptr() for g in grads)
                tab = self._tables.get(gi)
                if tab is None or tab[0] != key:
                    desc, chunks = C.adam_build([p.data for p in params], grads,
                                                [self.state[p]["exp_avg"] for p in params],
                                                [self.state[p]["exp_avg_sq"] for p in params], shadows)
                    tab = [key, desc, chunks, grads, gkey]
                    self._tables[gi] = tab
                elif tab[4] != gkey:
                    # The engine hands back fresh gradient tensors each step: rewrite only the
                    # table's gradient pointers on the device (no host round trip).
                    C.adam_patch_grads(tab[1], grads)
                    tab[3], tab[4] = grads, gkey
                C.adam_step(tab[1], tab[2], lr, b1, b2, eps, wd, step, 1.0, coef)
                # Shadows written by the kernel are current for the (unchanged) versions.
                for p, s in zip(params, shadows):
                    if s is not None:
                        p._dpfs_shadow = (p._version, s)
            else:
                grads = [p.grad for p in params]
                if coef is not None:
                    grads = [g * coef for g in grads]
                reference.adam_step([p.data for p in params], grads,
                                    [self.state[p]["exp_avg"] for p in params],
                                    [self.state[p]["exp_avg_sq"] for p in params], None,
                                    lr, b1, b2, eps, wd, step)
        return loss
