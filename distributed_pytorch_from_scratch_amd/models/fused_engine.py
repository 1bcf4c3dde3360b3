"""Explicit-schedule forward/backward of the whole TP decoder (the training fast path).

``Transformer.loss()`` runs through :class:`DecoderTrainFn`: one autograd Function whose
forward and hand-written backward call the kernel API directly (``ops.dispatch.K``: HIP
kernels on MI355X, the PyTorch oracle on CPU) in an explicit order.  Same math as the modular
layers (``parallel/layers.py``; the CPU/gloo equivalence tests run this path), but:

* **comm/compute overlap by ping-pong chunks.**  With TP > 1 the batch is split into
  ``chunks`` halves.  Every tensor-parallel all-reduce (row-parallel outputs in forward,
  column-parallel input-grads in backward) is launched ``async_op=True`` (RCCL runs on its own
  HIP stream) and waited only by the *next* segment of the *same* half, after the other half's
  segment has been enqueued on the compute stream:

      fwd  seg1(A) seg1(B) seg2(A)* seg2(B)* ...     seg1 = norm1,QKV,RoPE,attn,Wo -> AR
                                                     seg2 = *wait+bias+residual, norm2,
                                                            gate|up, SwiGLU, down -> AR
      bwd  b2(A) b2(B) b1(A)* b1(B)* ...             b2 = down/SwiGLU/gate|up grads -> AR(dh2)
                                                     b1 = *wait, norm2 bwd, Wo/attn/QKV grads
                                                          -> AR(dh)

  so each all-reduce is hidden behind the other half's GEMMs / attention (the reference issues
  every collective synchronously).  Inside a segment the weight-gradient GEMMs
  are issued after the all-reduce launch, so they overlap it too.
* fp32 weight-gradient accumulation across chunks inside the wgrad GEMM epilogue/reduce,
  norm/bias gradients from deterministic reductions (replicated params stay bitwise identical
  across TP ranks).
* bias + residual add fused in one kernel after the all-reduce; the logits all-gather is
  replaced by the vocab-parallel cross-entropy (one (M,3) stats all-gather per chunk).
* activations saved per chunk: x, normed inputs, roped QKV, attention output + LSE, gate|up,
  SwiGLU output — no (B,H,T,T) tensors.

Supported: RMSNorm blocks without sequence parallelism (the reference architecture and all
presets).  ``ModelArgs.sequence_parallel`` / LayerNorm models use the modular autograd path.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _ext
from ..ops import fp8 as F8
from ..ops import gemm_select as GS
from ..ops import reference
from ..ops.dispatch import K, emb_sort_ahead, emb_sort_take, shadow
from ..parallel import grad_sync as GSY
from ..parallel import process_manager as pm
from ..parallel import tp_comm


# A/B hook for tools/ab_attr.py, not a user switch: False keeps the two-pass CE at TP 1.
CE_ONE_PASS = True


def _ar(t: torch.Tensor):
    """Async TP all-reduce (RCCL or the xGMI peer-memory kernels: ``parallel/tp_comm.py``)."""
    p = pm.pgm
    if p is None or p.tp_size == 1:
        return None
    return tp_comm.all_reduce(t, async_op=True)


def _slot(ci: int, rows: int, cols: int, dt):
    """Staging buffer (xGMI communicator slot of chunk ``ci``) for a GEMM output that is
    all-reduced in place next (no copy-in); None -> the GEMM allocates.  The reduced tensor
    stays in the slot until the chunk's next staged GEMM, which comes after its consumers."""
    return tp_comm.staging(ci, (rows, cols), dt, "all_reduce")


def _wait(h):
    if h is not None:
        h.wait()


class _DeferredAdds:
    """Accumulation of the small fp32 gradients (bias / norm-weight column sums, embedding
    rows) over the chunks of a step.  The first chunk's kernel output is taken as the
    accumulator; later chunks' contributions are queued and added by one multi-tensor launch
    per flush (torch._foreach_add_) instead of one elementwise kernel each -- at TP 2 with two
    chunks that removes ~75 launches of ~5 us from the step (tools/tp_sim.py profile)."""

    def __init__(self):
        self.q = []

    def flush(self):
        while self.q:   # a target may appear once per launch (the foreach kernel runs lists in parallel)
            seen, now, later = set(), [], []
            for a, g in self.q:
                (later if id(a) in seen else now).append((a, g))
                seen.add(id(a))
            torch._foreach_add_([a for a, _ in now], [g for _, g in now])
            self.q = later


_DEFER = None   # the running backward's _DeferredAdds (the engines' backward is single-threaded)


def _defer_begin():
    global _DEFER
    _DEFER = _DeferredAdds()


def _defer_flush():
    if _DEFER is not None:
        _DEFER.flush()


def _defer_end():
    global _DEFER
    _defer_flush()
    _DEFER = None


def _addg(acc, g, view=None):
    """acc + g with the fp32 gradient accumulator ``acc`` (None: g is the first contribution; it
    lands in ``view``, the gradient's slot in the arena, unless it was written there already)."""
    if g is None:
        return acc
    if acc is None:
        if view is not None:
            if g is not view:
                view.copy_(g)
            return view
        return g.float() if g.dtype != torch.float32 else g   # fresh kernel output: take ownership
    if _DEFER is not None and g.dtype == torch.float32 and g.device == acc.device:
        _DEFER.q.append((acc, g))
        return acc
    return acc.add_(g)


class _Layer:
    """Parameter views of one DecoderLayer."""

    def __init__(self, layer):
        a, f = layer.attn, layer.ffn
        self.s1, self.s2 = layer.norm1.scale, layer.norm2.scale
        self.eps1, self.eps2 = layer.norm1.eps, layer.norm2.eps
        self.wqkv, self.bqkv = a.wqkv.weight, a.wqkv.bias
        self.wo, self.bo = a.wo.weight, a.wo.bias
        self.wgu, self.bgu = f.gate_up.weight, f.gate_up.bias
        self.wd, self.bd = f.down_proj.weight, f.down_proj.bias
        self.h, self.hd = a.num_local_heads, a.head_dim

    def params(self):
        return [self.s1, self.wqkv, self.bqkv, self.wo, self.bo, self.s2, self.wgu, self.bgu, self.wd, self.bd]


def _gate_up_weights(k, layers, W, want=None):
    """Per layer: whether its gate|up projection runs with SwiGLU in the GEMM epilogue
    (GS.swiglu_epilogue: the kernel reads the natural weight with its rows interleaved in
    64-row blocks and the backward returns natural-layout gradients, so nothing is copied)."""
    for L in layers:
        L.swi = GS.swiglu_epilogue(k, W(L.wgu), want)


def collect_params(model) -> List[Optional[torch.Tensor]]:
    ps = [model.embedding.weight]
    for layer in model.layers:
        ps += _Layer(layer).params()
    ps += [model.norm.scale, model.lm_head.weight, model.lm_head.bias]
    return ps


_LAYER_KEYS = ("s1", "wqkv", "bqkv", "wo", "bo", "s2", "wgu", "bgu", "wd", "bd")
_SP_REP = ("s1", "bo", "s2", "bd")   # replicated under SP (layers.py sequence_parallel_grad)


def arena_groups(model, layers, sp: bool):
    """Gradient groups in the order the engine's backward completes them (parallel/grad_sync
    GradArena): the head, the layers top-down (layer 0 after the embedding in the all-reduce
    engine, whose embedding gradient is produced before layer 0's weight gradients), and the
    embedding (+ final norm under SP, whose grad is summed over TP after the step)."""
    head = model.lm_head
    lay = lambda li: (f"L{li}", list(zip(_LAYER_KEYS, layers[li].params())))
    nL = len(layers)
    if sp:
        # the replicated gradients (norm scales, row-parallel biases: summed over TP after the
        # step) are stored together in one trailing range, "sprep", so that sum is one in-place
        # all-reduce of the arena (grad_sync.allreduce_sequence_parallel_grads)
        rep = lambda li: [((f"L{li}", k), q) for k, q in zip(_LAYER_KEYS, layers[li].params()) if k in _SP_REP]
        own = lambda li: (f"L{li}", [(k, q) for k, q in zip(_LAYER_KEYS, layers[li].params()) if k not in _SP_REP])
        return ([("head", [("lm_w", head.weight), ("lm_b", head.bias)])] + [own(li) for li in range(nL - 1, -1, -1)]
                + [("tail", [("emb", model.embedding.weight)])]
                + [("sprep", [x for li in range(nL - 1, -1, -1) for x in rep(li)] + [(("tail", "nf"), model.norm.scale)])])
    return ([("head", [("nf", model.norm.scale), ("lm_w", head.weight), ("lm_b", head.bias)])]
            + [lay(li) for li in range(nL - 1, 0, -1)] + [("emb", [("emb", model.embedding.weight)]), lay(0)])


def arena_begin(model, arena) -> bool:
    """Start of a backward over the arena.  True (the common case, ``zero_grad(set_to_none)``
    before the backward): the engine assigns the arena views as the parameters' ``.grad`` itself
    and returns no gradients to autograd (nothing is copied).  False: some ``.grad`` already
    holds an accumulated gradient -- a ``.grad`` that still aliases the arena is detached
    (cloned) first, since this backward overwrites the arena, and the gradients go back through
    autograd, which adds them."""
    params = [p for p in collect_params(model) if p is not None]
    if all(p.grad is None for p in params):
        return True
    lo, hi = arena.buf.data_ptr(), arena.buf.data_ptr() + 4 * arena.numel
    for p in params:
        if p.grad is not None and lo <= p.grad.data_ptr() < hi:
            p.grad = p.grad.clone()
    return False


def arena_end(model, grads, assign: bool):
    """The gradients to return from the engine's backward (see ``arena_begin``)."""
    if not assign:
        return grads
    for p, gr in zip(collect_params(model), grads):
        if p is not None and gr is not None:
            p.grad = gr
    return [None] * len(grads)


class DecoderTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, ids, pos, tgt, chunks: int, ignore_index: int, *params):
        dev = ids.device
        dt = model.act_dtype(dev)
        k = K(model.embedding.weight, model.act_dtype(model.embedding.weight.device))
        p = pm.pgm
        tp = 1 if p is None else p.tp_size
        B, T = ids.shape
        C = max(1, min(chunks, B))
        bounds = [(B * i) // C for i in range(C + 1)]
        layers = [_Layer(l) for l in model.layers]
        tab = model.rope_table(dev)
        emb = model.embedding
        head = model.lm_head
        vst = head.odim_start
        vvalid = max(0, min(model.vocab_size - vst, head.odim_partition))
        d = model.args.attn_dim
        recompute = bool(getattr(model.args, "recompute", False))

        W = lambda w: shadow(w, dt) if w is not None else None  # bf16 compute copies
        # fp8 step: one e4m3 copy (+ transposed copy) of every projection weight, looked up by
        # ops.gemm_select for the forward and the data-gradient GEMMs of this step
        f8map = F8.prepare([W(w) for L in layers for w in (L.wqkv, L.wo, L.wgu, L.wd)] + [W(model.lm_head.weight)]) \
            if getattr(model.args, "fp8", False) else None
        F8.activate(f8map)
        _gate_up_weights(k, layers, W, getattr(model.args, "swiglu_epilogue", None))
        st = []  # per-chunk saved state
        for c in range(C):
            b0, b1 = bounds[c], bounds[c + 1]
            ids_c = ids[b0:b1].reshape(-1).contiguous()
            x = k.embedding_fwd(ids_c, emb.weight, emb.vocab_st_idx, dt)
            # the embedding backward's sort, on a side stream beside the forward
            esort = emb_sort_ahead(ids_c, emb.vocab_st_idx, emb.weight.size(0)) if k is not reference else None
            st.append(dict(B=b1 - b0, ids=ids_c, esort=esort, pos=pos[b0:b1].reshape(-1).contiguous(),
                           tgt=tgt[b0:b1].reshape(-1).contiguous(), x=x, h=_ar(x), pend=None,
                           pend_bias=None, layers=[]))
        for li, L in enumerate(layers):
            # seg1: (wait + residual), norm1, QKV, RoPE, attention, Wo -> async all-reduce
            for ci, s in enumerate(st):
                _wait(s["h"])
                if s["pend"] is not None:   # residual epilogue of the previous layer fused into norm1
                    s["x"], h1, r1 = k.add_rmsnorm_fwd(s["pend"], s["pend_bias"], s["x"], L.s1, L.eps1)
                else:
                    h1, r1 = k.rmsnorm_fwd(s["x"], L.s1, L.eps1)
                x = s["x"]
                qkv = GS.gemm_nt_rope(k, h1, W(L.wqkv), L.bqkv, s["pos"], tab, 2 * L.h, L.hd)  # RoPE in the epilogue
                Mc = x.size(0)
                Bc = s["B"]
                q, kk, v = _split(qkv, Bc, T, L.h, L.hd)
                o, lse = k.attn_fwd(q, kk, v, 1.0 / math.sqrt(L.hd), True)
                o2 = o.view(Mc, L.h * L.hd)
                pout = GS.gemm_nt(k, o2, W(L.wo), None, out=_slot(ci, Mc, d, dt))
                s["layers"].append(dict(x=x, r1=r1, h1=h1, qkv=qkv, o=o, lse=lse))
                s["pend"], s["pend_bias"], s["h"] = pout, L.bo, _ar(pout)
            # seg2: wait + bias + residual, norm2, gate|up, SwiGLU, down -> async all-reduce
            for ci, s in enumerate(st):
                _wait(s["h"])
                x2, h2, r2 = k.add_rmsnorm_fwd(s["pend"], s["pend_bias"], s["x"], L.s2, L.eps2)
                gu, sw = GS.gate_up(k, h2, W(L.wgu), L.bgu, L.swi)   # SwiGLU in the epilogue
                qout = GS.gemm_nt(k, sw, W(L.wd), None, out=_slot(ci, sw.size(0), d, dt))
                s["layers"][-1].update(x2=x2, r2=r2, h2=h2, gu=gu, sw=sw)
                s["x"] = x2
                s["pend"], s["pend_bias"], s["h"] = qout, L.bd, _ar(qout)
                if recompute:          # keep only the layer input; the rest is rebuilt in backward
                    s["layers"][-1] = {"x": s["layers"][-1]["x"]}
        # head: residual, final norm, lm_head shard, vocab-parallel CE statistics.  TP 1 with a
        # unit loss gradient (engine.TrainStep): d logits is written in the same pass over the
        # logits as the statistics (k.ce_fused), so backward does not read them again.
        # the loss bookkeeping (lse, validity, running sums, the mean) in one kernel per chunk
        acc = torch.empty(2, device=dev, dtype=torch.float32)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        fuse_ce = CE_ONE_PASS and tp == 1 and getattr(model, "_ce_unit_grad", False) and hasattr(k, "ce_fused")
        if fuse_ce:
            gs_all, _ = k.ce_valid_scale(tgt.reshape(-1).contiguous(), ignore_index)
        row0 = 0
        for ci, s in enumerate(st):
            _wait(s["h"])
            xf, hf, rf = k.add_rmsnorm_fwd(s["pend"], s["pend_bias"], s["x"], model.norm.scale, model.norm.eps)
            logits = GS.gemm_nt(k, hf, W(head.weight), head.bias)
            stats = None
            if fuse_ce:
                gs = gs_all[row0:row0 + s["tgt"].numel()]
                db = torch.empty(logits.size(1), device=dev, dtype=torch.float32) if head.bias is not None else None
                stats = k.ce_fused(logits, s["tgt"], gs, vst, vvalid, db)
                if stats is not None:
                    s.update(ce_done=True, ce_db=db)
            if stats is None:
                stats = k.ce_fwd_stats(logits, s["tgt"], vst, vvalid)
            if tp > 1:
                allst = stats.new_empty((tp * stats.size(0), 3))
                dist.all_gather_into_tensor(allst, stats, group=p.tp_group)
                allst = allst.view(tp, -1, 3)
            else:
                allst = stats.unsqueeze(0)
            lse, valid = k.ce_finalize(allst, s["tgt"], ignore_index, acc, loss, ci == 0, ci == len(st) - 1)
            row0 += s["tgt"].numel()
            s.update(xf=xf, hf=hf, rf=rf, logits=logits, ce_lse=lse, valid=valid)
            del s["pend"], s["h"]
        ctx.model, ctx.st, ctx.layers, ctx.meta = model, st, layers, (T, dt, vst, vvalid, C, d)
        ctx.n_valid = acc[1]
        ctx.tab = tab
        ctx.nparams = len(params)
        ctx.recompute = recompute
        ctx.f8map = f8map
        F8.activate(None)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        model, st, layers = ctx.model, ctx.st, ctx.layers
        T, dt, vst, vvalid, C, d = ctx.meta
        k = K(model.embedding.weight, model.act_dtype(model.embedding.weight.device))
        head = model.lm_head
        W = lambda w: shadow(w, dt) if w is not None else None
        F8.activate(ctx.f8map)
        _defer_begin()
        tab = ctx.tab
        # d loss / d row (valid * gloss / n_valid, one native launch per chunk): only the CE
        # backward that did not run in the forward needs it
        nL = len(layers)
        # fp32 gradients: every one is written straight into its slot of the model's gradient
        # arena (parallel/grad_sync.GradArena; the first chunk's contribution in place, later
        # chunks accumulated), so the DP all-reduce runs on arena slices with no pack / copy
        arena = GSY.arena_for(model, arena_groups(model, layers, False), "tp")
        assign = arena_begin(model, arena)
        g = {"emb": None, "nf": None, "lm_w": None, "lm_b": None}
        gl = [dict() for _ in range(nL)]
        gname = {id(g): "head"}
        gname.update({id(gl[li]): f"L{li}" for li in range(nL)})
        V = lambda d_, key: arena.view(gname[id(d_)] if key != "emb" else "emb", key)

        def first(d_, key, like, n):
            """fp32 output buffer of a gradient kernel: the arena slot for the first chunk."""
            return V(d_, key) if d_.get(key) is None else like.new_empty(n, dtype=torch.float32)

        def tn(key_dict, key, dy, x):
            acc = key_dict.get(key)
            if acc is None:
                key_dict[key] = GS.gemm_tn(k, dy, x, V(key_dict, key))
            else:
                GS.gemm_tn(k, dy, x, acc, True)

        def tn_chunks(key_dict, key, pairs):
            """Weight gradient summed over the chunks ((dy, x) per chunk), issued after the
            last chunk's data-gradient GEMM of the phase: chunks go two at a time through
            GS.gemm_tn_pair (one split-K launch over both chunks' rows, one reduction)."""
            i = 0
            while i < len(pairs):
                if i + 1 < len(pairs):
                    (a0, b0), (a1, b1) = pairs[i], pairs[i + 1]
                    if key_dict.get(key) is None:
                        key_dict[key] = GS.gemm_tn_pair(k, a0, b0, a1, b1, V(key_dict, key), False)
                    else:
                        GS.gemm_tn_pair(k, a0, b0, a1, b1, key_dict[key], True)
                    i += 2
                else:
                    tn(key_dict, key, *pairs[i])
                    i += 1
            pairs.clear()

        def tn_multi(key_dict, groups):
            """Several weight gradients of one phase ((key, pairs) each): with one or two chunks,
            ONE grouped launch (GS.gemm_tn_group, timed against separate calls); else per key."""
            if all(len(pairs) == 1 for _, pairs in groups) or all(len(pairs) == 2 for _, pairs in groups):
                # (two chunks: each item's rows continue in the other chunk's buffers)
                items = []
                for key, pairs in groups:
                    acc = key_dict.get(key)
                    items.append((pairs[0][0], pairs[0][1], acc if acc is not None else V(key_dict, key),
                                  acc is not None) + (tuple(pairs[1]) if len(pairs) == 2 else ()))
                outs = GS.gemm_tn_group(k, items)
                for (key, pairs), o in zip(groups, outs):
                    key_dict[key] = o
                    pairs.clear()
                return
            for key, pairs in groups:
                tn_chunks(key_dict, key, pairs)

        def bias_acc(key_dict, key, dy, present):
            if present is None:
                return
            key_dict[key] = _addg(key_dict.get(key), k.bias_grad(dy), V(key_dict, key))

        # DP: each layer's gradients are marked complete as soon as the layer's backward is
        # done and go out as async all-reduces of contiguous arena slices (buckets of at least
        # the measured knee of the DP group's all-reduce curve, parallel/grad_sync), so they
        # overlap the remaining layers.
        pg = pm.pgm
        dp = pg.dp_size if pg is not None else 1
        dpb = GSY.DPBucketer(arena, pg.dp_group if dp > 1 else None, dp,
                             GSY.dp_bucket_bytes(pg.dp_group, gloss.device) if dp > 1 else 0,
                             before_launch=_defer_flush)
        dp_reduce = dpb.add

        # ---- head: CE backward in place over the logits, lm_head dgrad -> async AR
        lm_p = []
        for ci, s in enumerate(st):
            dl = s["logits"]
            if s.pop("ce_done", False):     # d logits (and its column sums) came with the forward
                db = s.pop("ce_db")
                # the forward assumed a unit loss gradient (loss(unit_grad=True)); a caller that
                # scaled the loss afterwards would get unscaled gradients.  Checking the value
                # costs a host sync, so it runs in the debug modes (DPFS_SYNC_DEBUG / NAN_CHECK)
                if ci == 0 and (_ext.debug_sync() or _ext.nan_check()) and not bool((gloss == 1).all()):
                    raise RuntimeError("loss(unit_grad=True) was differentiated with a non-unit gradient "
                                       f"({float(gloss.float().mean())}); call loss() without unit_grad when "
                                       "scaling the loss")
            else:
                gs = k.ce_grad_scale(s["valid"], gloss, ctx.n_valid)
                db = first(g, "lm_b", dl, dl.size(1)) if head.bias is not None else None
                k.ce_bwd(dl, s["tgt"], s["ce_lse"], gs, vst, vvalid, dl, db)    # + lm_head bias grad
            dh = GS.gemm_nn(k, dl, W(head.weight), out=_slot(ci, dl.size(0), d, dt))
            s["bh"] = _ar(dh)
            s["dpend"] = dh
            lm_p.append((dl, s["hf"]))
            if db is not None:
                g["lm_b"] = _addg(g["lm_b"], db, V(g, "lm_b"))
            del s["logits"]
        tn_chunks(g, "lm_w", lm_p)
        for s in st:
            _wait(s["bh"])
            Lt, Gt = layers[-1], gl[nL - 1]
            dbd = first(Gt, "bd", s["dpend"], s["dpend"].size(1)) if Lt.bd is not None else None
            dxf, dsf = k.rmsnorm_bwd(s["dpend"], s["xf"], model.norm.scale, s["rf"], None, dbd,
                                     dw_out=first(g, "nf", s["xf"], s["xf"].size(1)))
            if dbd is not None:   # bias grad of the last layer's down projection, same pass
                Gt["bd"] = _addg(Gt.get("bd"), dbd, V(Gt, "bd"))
                s["bd_done"] = True
            g["nf"] = _addg(g["nf"], dsf, V(g, "nf"))
            s["g"] = dxf            # grad wrt the last layer's output (residual stream)
            s["dpend"] = None
            del s["xf"], s["hf"]
        dp_reduce("head")

        def rebuild(L, li):
            """Activation recompute: re-run layer li's forward from its saved input up to the
            SwiGLU output.  The Wo all-reduce runs unstaged: each chunk's staging slot still
            holds the pending norm1 input-grad of layer li+1."""
            for s in st:
                a = s["layers"][li]
                a["h1"], a["r1"] = k.rmsnorm_fwd(a["x"], L.s1, L.eps1)
                a["qkv"] = GS.gemm_nt_rope(k, a["h1"], W(L.wqkv), L.bqkv, s["pos"], tab, 2 * L.h, L.hd)
                q, kk, v = _split(a["qkv"], s["B"], T, L.h, L.hd)
                a["o"], a["lse"] = k.attn_fwd(q, kk, v, 1.0 / math.sqrt(L.hd), True)
                pout = GS.gemm_nt(k, a["o"].view(a["qkv"].size(0), L.h * L.hd), W(L.wo), None)
                a["pout"], a["hh"] = pout, _ar(pout)
            for s in st:
                a = s["layers"][li]
                _wait(a.pop("hh"))
                a["x2"], a["h2"], a["r2"] = k.add_rmsnorm_fwd(a.pop("pout"), L.bo, a["x"], L.s2, L.eps2)
                a["gu"], a["sw"] = GS.gate_up(k, a["h2"], W(L.wgu), L.bgu, L.swi)

        # ---- layers, reversed
        for li in range(nL - 1, -1, -1):
            L, G = layers[li], gl[li]
            if ctx.recompute:
                rebuild(L, li)
            # b2: down / SwiGLU / gate|up grads -> AR(dh2)
            wd_p, wgu_p = [], []
            for ci, s in enumerate(st):
                if s["dpend"] is not None:     # finish the upper layer: wait, norm1 bwd, residual
                    _finish_norm1(k, s, layers[li + 1], gl[li + 1], li + 1, (G, L.bd), V=V)
                a = s["layers"][li]
                gq = s["g"]
                if not s.pop("bd_done", False):
                    bias_acc(G, "bd", gq, L.bd)
                wd_p.append((gq, a["sw"]))
                dbgu = first(G, "bgu", gq, a["gu"].size(1)) if L.bgu is not None else None
                # down dgrad with the SwiGLU backward (+ gate|up bias grad) in its epilogue
                dgu = GS.down_dgrad_swiglu(k, gq, W(L.wd), a["gu"], dbgu, L.swi)
                dh2 = GS.gemm_nn(k, dgu, W(L.wgu), out=_slot(ci, dgu.size(0), d, dt))
                s["bh"], s["dpend"] = _ar(dh2), dh2
                wgu_p.append((dgu, a["h2"]))
                if dbgu is not None:
                    G["bgu"] = _addg(G.get("bgu"), dbgu, V(G, "bgu"))
                del a["sw"], a["gu"]
            # With one chunk (no all-reduce to hide) the down / gate|up weight gradients wait for
            # the Wo / QKV ones: a layer's four go out as one grouped launch at the end of b1
            if C == 1:
                pend_w = [("wd", wd_p), ("wgu", wgu_p)]
            else:
                tn_multi(G, [("wd", wd_p), ("wgu", wgu_p)])        # under the chunks' all-reduces
                pend_w = []
            if li + 1 < nL:
                dp_reduce(f"L{li + 1}")         # layer li+1 is complete (its norm1 grad just landed)
            # b1: wait, norm2 bwd, Wo / attention / QKV grads -> AR(dh)
            wo_p, wqkv_p = [], []
            for ci, s in enumerate(st):
                a = s["layers"][li]
                _wait(s["bh"])
                dbo = first(G, "bo", s["dpend"], s["dpend"].size(1)) if L.bo is not None else None
                g2, ds2 = k.rmsnorm_bwd(s["dpend"], a["x2"], L.s2, a["r2"], s["g"], dbo,   # + residual grad, bo grad
                                        dw_out=first(G, "s2", a["x2"], a["x2"].size(1)))
                G["s2"] = _addg(G.get("s2"), ds2, V(G, "s2"))
                if dbo is not None:
                    G["bo"] = _addg(G.get("bo"), dbo, V(G, "bo"))
                do = GS.gemm_nn(k, g2, W(L.wo))
                wo_p.append((g2, a["o"].view(g2.size(0), -1)))
                Bc = s["B"]
                q, kk, v = _split(a["qkv"], Bc, T, L.h, L.hd)
                dqkv = torch.empty_like(a["qkv"])
                dq, dk, dv = _split(dqkv, Bc, T, L.h, L.hd)
                dbq = first(G, "bqkv", dqkv, dqkv.size(1)) if L.bqkv is not None else None
                # inverse RoPE fused into the dq/dk stores, the QKV bias grad into their epilogues
                bq_fused = k.attn_bwd(do.view(Bc, T, L.h, L.hd), q, kk, v, a["o"], a["lse"], 1.0 / math.sqrt(L.hd),
                                      True, dq, dk, dv, s["pos"], tab, dbias=dbq)
                dh = GS.gemm_nn(k, dqkv, W(L.wqkv), out=_slot(ci, dqkv.size(0), d, dt))
                s["bh"], s["dpend"] = _ar(dh), dh
                wqkv_p.append((dqkv, a["h1"]))
                if L.bqkv is not None:
                    G["bqkv"] = _addg(G.get("bqkv"), dbq if bq_fused else k.bias_grad(dqkv), V(G, "bqkv"))
                s["g"] = g2
                for key in ("x2", "r2", "h2", "qkv", "o", "lse"):
                    a.pop(key, None)
            if li > 0:
                tn_multi(G, pend_w + [("wo", wo_p), ("wqkv", wqkv_p)])
        # layer 0: the embedding gradient first, so its all-reduce (the largest DP bucket) runs
        # under layer 0's Wo / QKV weight-gradient GEMMs
        ev = arena.view("emb", "emb")
        for ci, s in enumerate(st):
            _finish_norm1(k, s, layers[0], gl[0], 0, V=V)
            # deterministic (sorted ids, no atomics): chunk 0 writes every row, the rest add
            perm, seg = emb_sort_take(s.pop("esort", None))
            k.embedding_bwd_sorted(s["g"], s["ids"], model.embedding.weight.size(0), model.embedding.vocab_st_idx,
                                   out=ev, accumulate=ci > 0, perm=perm, seg=seg)
        g["emb"] = ev
        dp_reduce("emb")
        tn_multi(gl[0], pend_w + [("wo", wo_p), ("wqkv", wqkv_p)])
        dp_reduce("L0")
        _defer_end()
        tp_comm.check()   # an xGMI barrier that timed out raises here (host-mapped flag, no sync)
        if dpb.finish():
            model._dpfs_dp_reduced = True   # DataParallelGradSync hooks skip this step
        ctx.st = None
        grads = [g["emb"]]
        for li, L in enumerate(layers):
            G = gl[li]
            grads += [G.get("s1"), G.get("wqkv"), G.get("bqkv") if L.bqkv is not None else None,
                      G.get("wo"), G.get("bo") if L.bo is not None else None, G.get("s2"), G.get("wgu"),
                      G.get("bgu") if L.bgu is not None else None, G.get("wd"),
                      G.get("bd") if L.bd is not None else None]
        grads += [g["nf"], g["lm_w"], g["lm_b"] if head.bias is not None else None]
        F8.activate(None)
        return (None, None, None, None, None, None) + tuple(arena_end(model, grads, assign))


def _finish_norm1(k, s, L, G, li, below=None, V=None):
    """Wait for the all-reduce of layer li's norm1 input-grad, run the norm1 backward and add
    it to the residual-stream grad (-> grad wrt layer li's input).  ``below`` = (grad dict,
    bias) of layer li-1's down projection: its bias grad (column sums of that residual grad)
    comes out of the same norm-backward pass.  ``V(dict, key)``: the gradient's arena slot."""
    a = s["layers"][li]
    _wait(s["bh"])
    db = None
    view = V if V is not None else (lambda d_, key: None)
    if below is not None and below[1] is not None:
        Gb = below[0]
        db = view(Gb, "bd") if Gb.get("bd") is None else None
        if db is None:
            db = s["g"].new_empty(s["g"].size(1), dtype=torch.float32)
    dw = view(G, "s1") if G.get("s1") is None else None      # the first chunk: straight into its slot
    s["g"], ds1 = k.rmsnorm_bwd(s["dpend"], a["x"], L.s1, a["r1"], s["g"], db, dw_out=dw)   # + residual grad
    if db is not None:
        below[0]["bd"] = _addg(below[0].get("bd"), db, view(below[0], "bd"))
        s["bd_done"] = True
    G["s1"] = _addg(G.get("s1"), ds1, view(G, "s1"))
    s["dpend"] = None
    for key in ("x", "r1", "h1"):
        a.pop(key, None)


def _split(qkv, B, T, h, hd):
    q = qkv[:, : h * hd].view(B, T, h, hd)
    k = qkv[:, h * hd: 2 * h * hd].view(B, T, h, hd)
    v = qkv[:, 2 * h * hd: 3 * h * hd].view(B, T, h, hd)
    return q, k, v


