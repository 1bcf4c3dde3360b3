"""LLaMA-style tensor-parallel decoder.

Reference parity: ``models/model.py`` (``Attention`` 49-78, ``FFN`` 81-95, ``DecoderLayer``
98-121, ``Transformer`` 124-158).  Same constructor signature, same ``reset_parameters()``
RNG order (embedding, then per layer wq, wk, wv, wo, gate, up, down, then lm_head), same
state-dict keys (``SURVEY.md`` §2.6) — so a reference checkpoint loads here and vice versa.

MI355X-first differences (same math):

* q|k|v and gate|up are fused column-parallel GEMMs (``FusedColumnParallelLinear``), which
  present the reference's separate ``wq/wk/wv`` and ``gate_proj/up_proj`` keys in
  ``state_dict``.
* attention is RoPE + causal flash attention on the packed QKV GEMM output (no ``(B,1,T,T)``
  mask, no ``(B,H,T,T)`` scores; ``model.py:73-77``); one RoPE table per model, indexed by
  position inside the kernel (``model.py:110,117-118`` kept one table per layer and gathered
  ``cos[position_ids]`` every layer).
* activations are bf16 on the GPU with fp32 master weights (explicit dtype policy instead of
  autocast); the CPU path runs fp32 end to end.
* heads / ffn columns / vocab may be partitioned unevenly (12 heads over TP=8).
* training uses a vocab-parallel cross-entropy on the local logit shard (``loss()``);
  ``forward()`` still returns full gathered ``(B, T, V)`` logits like the reference.
* optional Megatron sequence parallelism (``ModelArgs.sequence_parallel``).
"""
from __future__ import annotations

import os
from dataclasses import asdict
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import functional as Fn
from ..ops import reference as ref_ops
from ..parallel import comm_ops
from ..parallel import process_manager as pm
from ..parallel.cross_entropy import IGNORE_INDEX, vocab_parallel_cross_entropy
from ..parallel.layers import (ColumnParallelLinear, FusedColumnParallelLinear, LayerNorm,
                               ParallelVocabularyEmbedding, RMSNorm, RowParallelLinear,
                               attach_fused, partition_sizes)
from .config import ModelArgs, vocab_partition


def _tp():
    p = pm.pgm
    return (1, 0) if p is None else (p.tp_size, p.tp_rank)


def _make_norm(args: ModelArgs, sp: bool) -> nn.Module:
    if args.norm == "rmsnorm":
        return RMSNorm(args.attn_dim, args.norm_eps, sequence_parallel=sp)
    if args.norm == "layernorm":
        return LayerNorm(args.attn_dim, args.norm_eps, sequence_parallel=sp)
    raise ValueError(args.norm)


class Attention(nn.Module):
    def __init__(self, args: ModelArgs):
        super().__init__()
        n, r = _tp()
        d, H = args.attn_dim, args.num_heads
        assert d % H == 0
        self.attn_dim, self.num_heads, self.head_dim = d, H, d // H
        sizes = partition_sizes(d, n, self.head_dim)          # head-granular shards
        self.num_local_heads = sizes[r] // self.head_dim
        sp = args.sequence_parallel
        attach_fused(self, "wqkv", FusedColumnParallelLinear(
            d, [d, d, d], ["wq", "wk", "wv"], add_bias=args.bias, sizes=[sizes, sizes, sizes],
            sequence_parallel=sp))
        self.wo = RowParallelLinear(d, d, add_bias=args.bias, split_input=False, sizes=sizes,
                                    sequence_parallel=sp)

    def reset_parameters(self):
        self.wqkv.reset_parameters()
        self.wo.reset_parameters()

    def forward(self, x: torch.Tensor, positions: torch.Tensor, rope_table: torch.Tensor,
                B: int, T: int) -> torch.Tensor:
        qkv = self.wqkv(x)                                    # (B*T, 3*h_l*hd)
        h = self.num_local_heads
        o = Fn.causal_self_attention(qkv, positions, rope_table, B, T, h, h, self.head_dim, True)
        return self.wo(o)


class FFN(nn.Module):
    def __init__(self, args: ModelArgs):
        super().__init__()
        n, r = _tp()
        d, f = args.attn_dim, args.ffn_dim
        self.idim, self.hdim = d, f
        sizes = partition_sizes(f, n)
        sp = args.sequence_parallel
        attach_fused(self, "gate_up", FusedColumnParallelLinear(
            d, [f, f], ["gate_proj", "up_proj"], add_bias=args.bias, sizes=[sizes, sizes],
            sequence_parallel=sp))
        self.down_proj = RowParallelLinear(f, d, add_bias=args.bias, split_input=False, sizes=sizes,
                                           sequence_parallel=sp)

    def reset_parameters(self):
        self.gate_up.reset_parameters()
        self.down_proj.reset_parameters()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.down_proj(Fn.swiglu(self.gate_up(x)))


class DecoderLayer(nn.Module):
    def __init__(self, args: ModelArgs):
        super().__init__()
        self.head_dim = args.head_dim
        self.attn = Attention(args)
        self.ffn = FFN(args)
        self.norm1 = _make_norm(args, args.sequence_parallel)
        self.norm2 = _make_norm(args, args.sequence_parallel)

    def reset_parameters(self):
        self.attn.reset_parameters()
        self.ffn.reset_parameters()

    def forward(self, x, positions, rope_table, B: int, T: int):
        x = x + self.attn(self.norm1(x), positions, rope_table, B, T)
        x = x + self.ffn(self.norm2(x))
        return x


class Transformer(nn.Module):
    """``Transformer(attn_dim, ffn_dim, num_heads, num_layers, vocab_size, maxlen, rope_theta)``
    (reference signature, ``model.py:125``) or ``Transformer.from_args(ModelArgs)``."""

    def __init__(self, attn_dim: int = 512, ffn_dim: int = 2048, num_heads: int = 8,
                 num_layers: int = 12, vocab_size: int = 1024, maxlen: int = 2048,
                 rope_theta: float = 10000.0, args: Optional[ModelArgs] = None, **extra):
        super().__init__()
        if args is None:
            args = ModelArgs(attn_dim=attn_dim, ffn_dim=ffn_dim, num_heads=num_heads,
                             num_layers=num_layers, vocab_size=vocab_size, maxlen=maxlen,
                             rope_theta=rope_theta, **extra)
        self.args = args
        n, r = _tp()
        self.vocab_size = args.vocab_size
        self.padded_vocab_size = args.padded_vocab_size
        sp = args.sequence_parallel
        # Vocab shards (embedding rows = lm_head rows): the reference ranges, or balanced
        # against an uneven head split (config.vocab_partition).
        head_sizes = [w // args.head_dim for w in partition_sizes(args.attn_dim, n, args.head_dim)]
        vsizes = vocab_partition(args, head_sizes)
        self.embedding = ParallelVocabularyEmbedding(self.padded_vocab_size, args.attn_dim,
                                                     sequence_parallel=sp, sizes=vsizes)
        self.layers = nn.ModuleList([DecoderLayer(args) for _ in range(args.num_layers)])
        self.norm = _make_norm(args, sp)
        self.lm_head = ColumnParallelLinear(args.attn_dim, self.padded_vocab_size, add_bias=args.bias,
                                            gather_output=False, sizes=vsizes, sequence_parallel=sp)
        self.compute_dtype: Optional[torch.dtype] = None
        self._rope = {}
        self.use_fused_engine = True   # explicit-schedule fast path for loss()
        self.chunks: Optional[int] = None  # ping-pong chunks (default: 2 when TP > 1)

    @classmethod
    def from_args(cls, args: ModelArgs) -> "Transformer":
        return cls(args=args)

    # ---------------------------------------------------------------- init / utils ----
    def reset_parameters(self):
        self.embedding.reset_parameters()
        for layer in self.layers:
            layer.reset_parameters()
        self.lm_head.reset_parameters()

    def retain_grad(self):
        for _, p in self.named_parameters():
            if p.requires_grad:
                p.retain_grad()

    def set_compute_dtype(self, dtype: Optional[torch.dtype]):
        self.compute_dtype = dtype
        return self

    def act_dtype(self, device: torch.device) -> torch.dtype:
        """Activation dtype: explicit ``set_compute_dtype`` > bf16 on the GPU (the MFMA kernels
        are bf16-in / fp32-accumulate) > the reference's ``DTYPE`` env var (``model.py:153``)
        on the CPU oracle path > the parameter dtype."""
        if self.compute_dtype is not None:
            return self.compute_dtype
        if device.type == "cuda":
            return torch.bfloat16
        env = os.environ.get("DTYPE")
        if env in ("bfloat16", "float32"):
            return torch.bfloat16 if env == "bfloat16" else torch.float32
        return self.embedding.weight.dtype

    def rope_table(self, device) -> torch.Tensor:
        key = str(device)
        t = self._rope.get(key)
        if t is None:
            t = ref_ops.rope_table(self.args.maxlen, self.args.head_dim, self.args.rope_theta).to(device)
            self._rope[key] = t
        return t

    def num_parameters(self, global_count: bool = True) -> int:
        """Parameter count; ``global_count`` reconstructs the full model size from the shards
        (the reference prints the local shard count, ``train.py:71-74``)."""
        local = sum(p.numel() for p in self.parameters())
        p = pm.pgm
        if not global_count or p is None or p.tp_size == 1:
            return local
        replicated = sum(p_.numel() for n_, p_ in self.named_parameters() if _is_replicated(n_))
        t = torch.tensor([local - replicated], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t, group=p.tp_group)
        return int(t.item()) + replicated

    # ---------------------------------------------------------------------- forward ----
    def _trunk(self, input_ids: torch.Tensor, position_ids: torch.Tensor):
        B, T = input_ids.shape
        dt = self.act_dtype(input_ids.device)
        self.embedding.out_dtype = dt
        x = self.embedding(input_ids)
        x = x.reshape(-1, x.size(-1))
        if x.dtype != dt:
            x = x.to(dt)
        positions = position_ids.reshape(-1)
        tab = self.rope_table(input_ids.device)
        assert int(T) <= self.args.maxlen, f"sequence length {T} > maxlen {self.args.maxlen}"
        for layer in self.layers:
            x = layer(x, positions, tab, B, T)
        return self.norm(x), B, T

    def _lm_head_local(self, h: torch.Tensor) -> torch.Tensor:
        w = self.lm_head
        from ..parallel.linear_fn import column_parallel_linear
        return column_parallel_linear(h, w.weight, w.bias, w.sequence_parallel, True)

    def forward(self, input_ids: torch.Tensor, position_ids: torch.Tensor) -> torch.Tensor:
        """Full ``(B, T, vocab_size)`` logits on every rank (reference contract)."""
        h, B, T = self._trunk(input_ids, position_ids)
        logits = self._lm_head_local(h)
        logits = comm_ops.Gather.apply(logits, self.lm_head.sizes)
        return logits[..., : self.vocab_size].reshape(B, T, self.vocab_size)

    def fused_supported(self) -> bool:
        """The explicit-schedule engines cover RMSNorm blocks, with (``fused_engine_sp``) or
        without (``fused_engine``) sequence parallelism; LayerNorm models use the modular path."""
        return self.args.norm == "rmsnorm" and self.use_fused_engine

    def overlap_chunks(self) -> int:
        p = pm.pgm
        if self.chunks is not None:
            return self.chunks
        return 2 if (p is not None and p.tp_size > 1) else 1

    def loss(self, input_ids: torch.Tensor, position_ids: torch.Tensor, target_ids: torch.Tensor,
             ignore_index: int = IGNORE_INDEX, unit_grad: bool = False) -> torch.Tensor:
        """Mean next-token CE via the vocab-parallel cross-entropy (no logits all-gather).

        Runs the explicit-schedule engine (``models/fused_engine.py``: ping-pong chunks with
        all-reduces overlapped by the other chunk's compute) when supported, else the modular
        autograd path.  ``unit_grad``: the caller differentiates the returned loss with a unit
        gradient (``loss.backward()``, as ``engine.TrainStep`` does), so at TP 1 the engine may
        compute d logits in the forward, in the same pass over the logits as the loss."""
        if self.fused_supported():
            self._ce_unit_grad = bool(unit_grad)
            from .fused_engine import DecoderTrainFn, collect_params
            assert input_ids.size(1) <= self.args.maxlen
            p = pm.pgm
            fn = DecoderTrainFn
            if self.args.sequence_parallel and p is not None and p.tp_size > 1:
                from .fused_engine_sp import DecoderTrainFnSP as fn
            return fn.apply(self, input_ids, position_ids, target_ids.reshape(input_ids.shape),
                            self.overlap_chunks(), ignore_index, *collect_params(self))
        h, B, T = self._trunk(input_ids, position_ids)
        logits = self._lm_head_local(h)
        st = self.lm_head.odim_start
        valid = max(0, min(self.vocab_size - st, logits.size(-1)))
        return vocab_parallel_cross_entropy(logits, target_ids.reshape(-1), st, valid, ignore_index,
                                            inplace_backward=True)


def _is_replicated(name: str) -> bool:
    """Parameters that are identical on every TP rank (not sharded)."""
    return (name.endswith("scale") or name.endswith("norm1.weight") or name.endswith("norm2.weight")
            or name.endswith("norm.weight") or name.endswith("norm1.bias") or name.endswith("norm2.bias")
            or name.endswith("norm.bias") or name.endswith("wo.bias") or name.endswith("down_proj.bias"))


def sequence_parallel_grad_params(model: nn.Module):
    return [p for p in model.parameters() if getattr(p, "sequence_parallel_grad", False)]


def build_model(args: ModelArgs, device, seed: Optional[int] = None) -> Transformer:
    if seed is not None:
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)
    m = Transformer.from_args(args).to(device)
    m.reset_parameters()
    return m
