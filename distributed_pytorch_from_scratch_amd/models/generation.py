"""KV-cached autoregressive decoding for the tensor-parallel Transformer.

The reference decodes greedily by re-running the whole prefix every token (``test.py:144-150``:
O(T²·L) work per token, no cache). This module keeps each layer's post-RoPE keys and values
for the local head shard. It prefills the prompt with the causal flash-attention kernel, then
decodes one token per step: one query row against the cached keys. TP works as in training:
heads are sharded, the row-parallel projections all-reduce, and the vocab-sharded logits are
all-gathered before the argmax. Every rank therefore picks the same token.

``generate(model, prompt, ...)`` returns the prompt followed by the generated ids.
``logits_step`` exposes the last-position logits (tests compare it against the full recompute).
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch

from ..ops.dispatch import K
from ..parallel import comm_ops


class KVCache:
    """Per-layer key/value buffers ``(B, T_max, H_local, hd)`` in the activation dtype."""

    def __init__(self, n_layers: int, B: int, t_max: int, h_local: int, hd: int, dtype, device):
        self.k = [torch.empty(B, t_max, h_local, hd, dtype=dtype, device=device) for _ in range(n_layers)]
        self.v = [torch.empty(B, t_max, h_local, hd, dtype=dtype, device=device) for _ in range(n_layers)]
        self.len = 0
        self.t_max = t_max


def _attention_step(layer, x2d, positions, tab, cache: KVCache, li: int, B: int, T: int):
    attn = layer.attn
    h, hd = attn.num_local_heads, attn.head_dim
    qkv = attn.wqkv(x2d)                                     # (B*T, 3*h*hd)
    k_ = K(qkv)
    k_.rope_(qkv, positions, tab, 2 * h, hd, False)
    q = qkv[:, : h * hd].view(B, T, h, hd)
    kk = qkv[:, h * hd: 2 * h * hd].view(B, T, h, hd)
    v = qkv[:, 2 * h * hd:].view(B, T, h, hd)
    t0 = cache.len
    cache.k[li][:, t0:t0 + T] = kk
    cache.v[li][:, t0:t0 + T] = v
    scale = 1.0 / math.sqrt(hd)
    if t0 == 0:
        # prefill: causal flash attention over the prompt
        o, _ = k_.attn_fwd(q, kk, v, scale, True)
    else:
        # decode: T new queries (T == 1 in greedy decode) against every cached key
        keys = cache.k[li][:, : t0 + T].float()             # (B, S, h, hd)
        vals = cache.v[li][:, : t0 + T].float()
        s = torch.einsum("bthd,bshd->bhts", q.float(), keys) * scale
        if T > 1:
            S = t0 + T
            mask = torch.ones(T, S, dtype=torch.bool, device=s.device).triu(S - T + 1)
            s = s.masked_fill(mask, float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("bhts,bshd->bthd", p, vals).to(q.dtype)
    return attn.wo(o.reshape(B * T, h * hd))


@torch.inference_mode()
def logits_step(model, ids: torch.Tensor, cache: KVCache) -> torch.Tensor:
    """Feed ``ids`` (B, T) at positions cache.len.., return (B, vocab) logits of the last one."""
    B, T = ids.shape
    dev = ids.device
    dt = model.act_dtype(dev)
    assert cache.len + T <= cache.t_max <= model.args.maxlen
    model.embedding.out_dtype = dt
    x = model.embedding(ids).reshape(B * T, -1).to(dt)
    positions = torch.arange(cache.len, cache.len + T, device=dev).repeat(B)
    tab = model.rope_table(dev)
    for li, layer in enumerate(model.layers):
        x = x + _attention_step(layer, layer.norm1(x), positions, tab, cache, li, B, T)
        x = x + layer.ffn(layer.norm2(x))
    cache.len += T
    h = model.norm(x.view(B, T, -1)[:, -1].contiguous())
    logits = model._lm_head_local(h)
    logits = comm_ops.Gather.apply(logits, model.lm_head.sizes)
    return logits[..., : model.vocab_size].float()


@torch.inference_mode()
def generate(model, prompt: torch.Tensor, max_new_tokens: int, eos_id: Optional[int] = None,
             max_len: Optional[int] = None) -> List[List[int]]:
    """Greedy decoding with a KV cache. ``prompt`` (B, T0) int64. Returns, per sequence, the
    prompt plus the generated ids. A sequence stops after emitting ``eos_id`` (kept in the
    output) or when the total length reaches ``max_len`` (default: model maxlen)."""
    B, T0 = prompt.shape
    dev = prompt.device
    t_max = min(model.args.maxlen, max_len or model.args.maxlen, T0 + max_new_tokens)
    attn0 = model.layers[0].attn
    cache = KVCache(len(model.layers), B, t_max, attn0.num_local_heads, attn0.head_dim,
                    model.act_dtype(dev), dev)
    out = [list(map(int, row)) for row in prompt.tolist()]
    done = [False] * B
    if max_new_tokens <= 0 or T0 >= t_max:
        return out
    logits = logits_step(model, prompt, cache)
    n_gen = 0
    while True:
        nxt = logits.argmax(-1)
        n_gen += 1
        for b, t in enumerate(nxt.tolist()):
            if not done[b]:
                out[b].append(int(t))
                done[b] = eos_id is not None and int(t) == eos_id
        if all(done) or n_gen >= max_new_tokens or cache.len >= t_max:
            return out
        logits = logits_step(model, nxt.view(B, 1), cache)
