"""KV-cached autoregressive decoding for the tensor-parallel Transformer.

The reference decodes greedily by re-running the whole prefix every token (``test.py:144-150``:
O(T²·L) work per token, no cache). This module keeps each layer's post-RoPE keys and values
for the local head shard:

* prefill: the prompt goes through the causal flash-attention kernel and fills cache rows
  ``[0, T0)``;
* decode: one token per sequence per step.  The step is written against DEVICE state only —
  the cache length ``cache.len_t`` (int32) and the position ids ``pos`` live on the GPU, the
  new key/value rows are appended at ``len_t`` (``kv_append``), the single-query split-K
  attention kernel (``attn_decode``, csrc/kernels/decode.hip) reads ``len_t`` itself, and
  ``step_advance`` bumps ``len_t`` / ``pos`` at the end — so at TP = 1 the whole step (about
  20 kernels per layer) is captured once in a HIP graph and replayed per token, instead of being
  re-launched from Python.  With TP > 1 the same step runs eagerly (the row-parallel outputs
  are all-reduced and the vocab-sharded logits all-gathered, so every rank picks the same
  token).  ``DPFS_DECODE_GRAPH=0`` forces the eager step.

``generate(model, prompt, ...)`` returns the prompt followed by the generated ids.
``logits_step`` exposes the last-position logits (tests compare it against the full recompute).
"""
from __future__ import annotations

import math
import os
import weakref
from typing import List, Optional

import torch

# decode steps captured per HIP graph replay (the host reads the tokens / checks EOS once per
# replay; profiles/r2_decode_bench.jsonl)
_GRAPH_STEPS = 8

from ..ops import gemm_select as GS
from ..ops.dispatch import K, shadow
from ..parallel import comm_ops
from ..parallel import process_manager as pm
from ..parallel import tp_comm


class KVCache:
    """Per-layer key/value buffers ``(B, T_max, H_local, hd)`` in the activation dtype."""

    def __init__(self, n_layers: int, B: int, t_max: int, h_local: int, hd: int, dtype, device):
        self.k = [torch.empty(B, t_max, h_local, hd, dtype=dtype, device=device) for _ in range(n_layers)]
        self.v = [torch.empty(B, t_max, h_local, hd, dtype=dtype, device=device) for _ in range(n_layers)]
        self.len = 0                      # host view (prefill / multi-token steps)
        self.len_t = torch.zeros(1, dtype=torch.int32, device=device)   # device view (decode steps)
        self.t_max = t_max

    def sync_device_len(self):
        self.len_t.fill_(self.len)


def _attention_step(layer, x2d, positions, tab, cache: KVCache, li: int, B: int, T: int):
    """Multi-token step (prefill, or T > 1 continuation) with host-side cache bookkeeping."""
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
        # T new queries against every cached key (continuation chunk)
        keys = cache.k[li][:, : t0 + T].float()             # (B, S, h, hd)
        vals = cache.v[li][:, : t0 + T].float()
        s = torch.einsum("bthd,bshd->bhts", q.float(), keys) * scale
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
    if T == 1 and cache.len > 0:
        cache.sync_device_len()
        pos = torch.full((B,), cache.len, dtype=torch.int64, device=dev)
        _, logits = decode_step(model, ids, pos, cache)
        cache.len += 1
        return logits
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


def decode_step(model, ids: torch.Tensor, pos: torch.Tensor, cache: KVCache):
    """One token per sequence (``ids`` (B, 1), ``pos`` (B,) int64 = cache.len_t) against the
    cache; advances ``cache.len_t`` and ``pos`` on the device.  Returns (next ids (B,),
    logits (B, vocab) fp32).  Touches no host state: graph-capturable."""
    from .fused_engine import _Layer
    if model.args.norm != "rmsnorm":
        return _decode_step_modules(model, ids, pos, cache)
    B = ids.size(0)
    dev = ids.device
    dt = model.act_dtype(dev)
    k = K(model.embedding.weight, dt)
    W = lambda w: shadow(w, dt) if w is not None else None
    model.embedding.out_dtype = dt
    x = model.embedding(ids).reshape(B, -1).to(dt)
    tab = model.rope_table(dev)
    pend = pend_bias = None
    small = B <= 16

    def proj(a, w, bias=None, swiglu=False):
        if small:   # MFMA GEMV-class kernel, SwiGLU fused into the down projection's operand
            return GS.small_nt(k, a, w, bias, swiglu)
        return GS.gemm_nt(k, k.swiglu_fwd(a) if swiglu else a, w, bias)
    # Per layer: [bias + residual +] RMSNorm (one kernel), QKV projection, RoPE + append of
    # k/v at len (one kernel), split-K decode attention, Wo projection, bias + residual +
    # RMSNorm, gate|up projection, SwiGLU + down projection (its bias + residual fold into the
    # next layer's norm).
    for li, layer in enumerate(model.layers):
        L = _Layer(layer)
        if pend is None:
            h1, _ = k.rmsnorm_fwd(x, L.s1, L.eps1)
        else:
            x, h1, _ = k.add_rmsnorm_fwd(pend, pend_bias, x, L.s1, L.eps1)
        qkv = proj(h1, W(L.wqkv), L.bqkv)
        if L.hd % 16 == 0:
            k.rope_append(qkv, pos, tab, cache.k[li], cache.v[li], cache.len_t)
        else:
            k.rope_(qkv, pos, tab, 2 * L.h, L.hd, False)
            k.kv_append(qkv, cache.k[li], cache.v[li], cache.len_t)
        o = k.attn_decode(qkv, cache.k[li], cache.v[li], cache.len_t, 1.0 / math.sqrt(L.hd))
        pout = proj(o, W(L.wo))
        tp_comm.all_reduce(pout, async_op=False)
        x, h2, _ = k.add_rmsnorm_fwd(pout, L.bo, x, L.s2, L.eps2)
        pend, pend_bias = proj(proj(h2, W(L.wgu), L.bgu), W(L.wd), swiglu=True), L.bd
        tp_comm.all_reduce(pend, async_op=False)
    _, hfin, _ = k.add_rmsnorm_fwd(pend, pend_bias, x, model.norm.scale, model.norm.eps)
    logits = proj(hfin, W(model.lm_head.weight), model.lm_head.bias)
    logits = comm_ops.Gather.apply(logits, model.lm_head.sizes)[..., : model.vocab_size].float()
    nxt = logits.argmax(-1)
    K(pos).step_advance(cache.len_t, pos)
    return nxt, logits


def _decode_step_modules(model, ids: torch.Tensor, pos: torch.Tensor, cache: KVCache):
    """decode_step through the nn.Module layers (any norm type, e.g. the LayerNorm variant)."""
    B = ids.size(0)
    dev = ids.device
    dt = model.act_dtype(dev)
    model.embedding.out_dtype = dt
    x = model.embedding(ids).reshape(B, -1).to(dt)
    tab = model.rope_table(dev)
    for li, layer in enumerate(model.layers):
        attn = layer.attn
        h, hd = attn.num_local_heads, attn.head_dim
        qkv = attn.wqkv(layer.norm1(x))                      # (B, 3*h*hd)
        k_ = K(qkv)
        k_.rope_(qkv, pos, tab, 2 * h, hd, False)
        k_.kv_append(qkv, cache.k[li], cache.v[li], cache.len_t)
        x = x + attn.wo(k_.attn_decode(qkv, cache.k[li], cache.v[li], cache.len_t, 1.0 / math.sqrt(hd)))
        x = x + layer.ffn(layer.norm2(x))
    logits = model._lm_head_local(model.norm(x))
    logits = comm_ops.Gather.apply(logits, model.lm_head.sizes)[..., : model.vocab_size].float()
    nxt = logits.argmax(-1)
    K(pos).step_advance(cache.len_t, pos)
    return nxt, logits


class DecodeGraph:
    """``nsteps`` decode steps captured as one HIP graph (static ids / pos / output buffers):
    step s writes its next ids into ``outs[s]`` and feeds them to step s + 1 on the device, so
    the host reads the tokens back (and checks EOS) once per replay instead of once per token
    (that round trip, ~90 us, was idle GPU time in every step)."""

    def __init__(self, model, cache: KVCache, B: int, nsteps: int = 1):
        dev = cache.len_t.device
        self.cache = cache
        self.nsteps = nsteps
        self.ids = torch.zeros(B, 1, dtype=torch.int64, device=dev)
        self.pos = torch.zeros(B, dtype=torch.int64, device=dev)
        self.outs = torch.zeros(nsteps, B, dtype=torch.int64, device=dev)
        saved = cache.len_t.clone()
        # Warm-up off the capture (first-call GEMM choices, allocator pools).  It appends a row
        # at len_t, which the first real step rewrites before anything reads it.
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.pos.copy_(cache.len_t.long().expand(B))
            decode_step(model, self.ids, self.pos, cache)
        torch.cuda.current_stream().wait_stream(s)
        cache.len_t.copy_(saved)
        _graph_rng_state_normal(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for i in range(nsteps):
                nxt, self.logits = decode_step(model, self.ids, self.pos, cache)
                self.outs[i].copy_(nxt)
                if i + 1 < nsteps:
                    self.ids.copy_(nxt.view(-1, 1))
        self.out = self.outs[nsteps - 1]
        cache.len_t.copy_(saved)

    def step(self, ids: torch.Tensor) -> torch.Tensor:
        """Feed ids (B,) at the cache's device length; returns the next ids of every captured
        step (nsteps, B) (device); the cache advances by nsteps rows."""
        self.ids.copy_(ids.view(-1, 1))
        self.graph.replay()
        return self.outs


_RNG_GRAPH_STATE = {}


def _graph_rng_state_normal(dev) -> None:
    """The CUDA generator's graph-safe RNG state is allocated when the first graph registers with
    the generator (and freed when the last one is destroyed); allocated under inference mode
    (this module's decode paths) those tensors are inference tensors, and every later capture
    outside inference mode (engine.GraphTrainStep) fails on their in-place update.  So a
    one-op graph built with inference mode off is kept alive for the process: the state is
    allocated once, as normal tensors, before the first decode capture."""
    if dev.index in _RNG_GRAPH_STATE:
        return
    with torch.inference_mode(False):
        x = torch.zeros(1, device=dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            x.add_(1)
    _RNG_GRAPH_STATE[dev.index] = (g, x)


def _use_graph(dev) -> bool:
    p = pm.pgm
    return (dev.type == "cuda" and os.environ.get("DPFS_DECODE_GRAPH", "1") != "0"
            and (p is None or p.tp_size == 1))


_SESSIONS = {}   # (id(model), B, t_max, device) -> KV cache + captured decode graphs


def _session(model, B: int, t_max: int, dev):
    """The KV cache and decode graphs for this (model, batch, length): reused by the next
    generate() call of the same shape, so serving pays the graph capture once.  Reused only
    while it is the same live model object and no parameter changed since the capture (the
    graphs hold the bf16 weight copies of that version); otherwise rebuilt.  One kept shape
    per model, and only caches up to DPFS_DECODE_SESSION_MAX_GB (default 16) are kept;
    ``clear_sessions()`` frees them."""
    attn0 = model.layers[0].attn
    key = (id(model), B, t_max, str(dev))
    vers = tuple(p._version for p in model.parameters())
    ent = _SESSIONS.get(key)
    if ent is not None and ent["model"]() is model and ent["vers"] == vers:
        ent["cache"].len = 0
        return ent["cache"], ent["graphs"]
    cache = KVCache(len(model.layers), B, t_max, attn0.num_local_heads, attn0.head_dim, model.act_dtype(dev), dev)
    graphs = {}
    kv_bytes = sum(t.numel() * t.element_size() for t in cache.k + cache.v)
    keep_gb = float(os.environ.get("DPFS_DECODE_SESSION_MAX_GB", "16"))
    if _use_graph(dev) and kv_bytes <= keep_gb * 2 ** 30:
        for k in [k for k, e in _SESSIONS.items() if e["model"]() is None or k[0] == id(model)]:
            del _SESSIONS[k]          # dead models, and other shapes of this one
        _SESSIONS[key] = {"model": weakref.ref(model), "vers": vers, "cache": cache, "graphs": graphs}
    return cache, graphs


def clear_sessions():
    """Drop every kept KV cache and decode graph (frees their device memory)."""
    _SESSIONS.clear()


@torch.inference_mode()
def generate(model, prompt: torch.Tensor, max_new_tokens: int, eos_id: Optional[int] = None,
             max_len: Optional[int] = None) -> List[List[int]]:
    """Greedy decoding with a KV cache. ``prompt`` (B, T0) int64. Returns, per sequence, the
    prompt plus the generated ids. A sequence stops after emitting ``eos_id`` (kept in the
    output) or when the total length reaches ``max_len`` (default: model maxlen)."""
    B, T0 = prompt.shape
    dev = prompt.device
    t_max = min(model.args.maxlen, max_len or model.args.maxlen, T0 + max_new_tokens)
    cache, graphs = _session(model, B, t_max, dev)
    out = [list(map(int, row)) for row in prompt.tolist()]
    done = [False] * B
    if max_new_tokens <= 0 or T0 >= t_max:
        return out
    nxt = logits_step(model, prompt, cache).argmax(-1)
    cache.sync_device_len()
    pos = torch.full((B,), cache.len, dtype=torch.int64, device=dev)
    chunk = _GRAPH_STEPS
    n_gen = 0

    def emit(row) -> bool:
        """Append one step's ids; True when generation is finished."""
        nonlocal n_gen
        n_gen += 1
        for b, t in enumerate(row):
            if not done[b]:
                out[b].append(int(t))
                done[b] = eos_id is not None and int(t) == eos_id
        return all(done) or n_gen >= max_new_tokens or cache.len >= t_max

    if emit(nxt.tolist()):
        return out
    while True:
        if _use_graph(dev):
            # S steps per replay while S more tokens are wanted and the cache has room for them
            S = chunk if (max_new_tokens - n_gen >= chunk and cache.len + chunk <= t_max) else 1
            g = graphs.get(S)
            if g is None:
                g = graphs[S] = DecodeGraph(model, cache, B, S)
            g.pos.fill_(cache.len)
            outs = g.step(nxt)
            rows = outs.tolist()
            nxt = g.out
            for row in rows:
                cache.len += 1
                if emit(row):
                    return out
        else:
            nxt, _ = decode_step(model, nxt.view(B, 1), pos, cache)
            cache.len += 1
            if emit(nxt.tolist()):
                return out
