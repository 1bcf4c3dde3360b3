"""Explicit-schedule training step with Megatron sequence parallelism (``--sp``).

Same math and kernels as :mod:`.fused_engine`, but the residual stream between the
tensor-parallel blocks is sharded over the TP group by token rows (rank r holds rows
``[r*M/n, (r+1)*M/n)`` of every chunk):

* forward, per block: ``RS`` (reduce-scatter) of the row-parallel output replaces the
  all-reduce; bias + residual + RMSNorm run on the local rows only; an ``AG`` (all-gather) of
  the normed rows feeds the next column-parallel GEMM;
* backward, mirrored: the column-parallel input-gradient is reduce-scattered, the norm
  backward runs on the local rows, and the residual gradient is all-gathered for the
  row-parallel dgrad / wgrad.

The bytes on the wire equal the all-reduce version (RS + AG = one all-reduce), but every
per-token elementwise op (norms, residual adds) does 1/n of the work.  At TP = 8 on the
GPT-2-small bench shape that removes ~19 ms/step of replicated norm work (24 add+RMSNorm
forwards at 537 us and 24 norm backwards at 368 us for 262k rows, profiles/).  The gradients
of the replicated parameters (norm scales, row-parallel biases) come out as per-rank partial
sums over the local rows, exactly like the modular SP layers; ``TrainStep`` sums them over
the TP group (``allreduce_sequence_parallel_grads``), so they end bitwise identical on every
rank.

Chunks (ping-pong) and the per-phase interleaving work as in the all-reduce engine: each
collective is launched async and waited by the next phase of the same chunk, after the other
chunk's phase has been enqueued.  Reference parity: the reference has no sequence
parallelism; the modular layers' SP path (``parallel/comm_ops.py``
``ScatterSeq`` / ``GatherSeq``) computes the same function.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from ..ops import fp8 as F8
from ..ops import gemm_select as GS
from ..ops import reference
from ..ops.dispatch import K, emb_sort_ahead, emb_sort_take, shadow
from ..parallel import grad_sync as GSY
from ..parallel import process_manager as pm
from ..parallel import tp_comm
from .fused_engine import (_Layer, arena_begin, arena_end, arena_groups, _addg, _defer_begin, _defer_end, _defer_flush,
                           _gate_up_weights, _split, _wait)


def _rs(full: torch.Tensor, n: int):
    """Reduce-scatter rows of ``full`` -> (local rows, work)."""
    out = full.new_empty((full.size(0) // n,) + tuple(full.shape[1:]))
    return out, tp_comm.reduce_scatter(out, full, async_op=True)


def _slot(ci: int, rows: int, cols: int, dt):
    """Staging buffer (xGMI communicator slot of chunk ``ci``) for a GEMM output that feeds a
    reduce-scatter, so the collective reads it in place; None -> the GEMM allocates."""
    return tp_comm.staging(ci, (rows, cols), dt, "reduce_scatter")


def _ag(part: torch.Tensor, n: int):
    """All-gather rows of ``part`` -> (full rows, work)."""
    out = part.new_empty((part.size(0) * n,) + tuple(part.shape[1:]))
    return out, tp_comm.all_gather(out, part, async_op=True)


class DecoderTrainFnSP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, ids, pos, tgt, chunks: int, ignore_index: int, *params):
        dev = ids.device
        dt = model.act_dtype(dev)
        k = K(model.embedding.weight, model.act_dtype(model.embedding.weight.device))
        p = pm.pgm
        n = p.tp_size
        B, T = ids.shape
        C = max(1, min(chunks, B))
        bounds = [(B * i) // C for i in range(C + 1)]
        layers = [_Layer(l) for l in model.layers]
        tab = model.rope_table(dev)
        emb, head = model.embedding, model.lm_head
        d = model.args.attn_dim
        recompute = bool(getattr(model.args, "recompute", False))
        vst = head.odim_start
        vvalid = max(0, min(model.vocab_size - vst, head.odim_partition))
        W = lambda w: shadow(w, dt) if w is not None else None
        # fp8 step: one e4m3 copy (+ transposed copy) of every projection weight, looked up by
        # ops.gemm_select for the forward and the data-gradient GEMMs of this step
        f8map = F8.prepare([W(w) for L in layers for w in (L.wqkv, L.wo, L.wgu, L.wd)] + [W(model.lm_head.weight)]) \
            if getattr(model.args, "fp8", False) else None
        F8.activate(f8map)
        _gate_up_weights(k, layers, W, getattr(model.args, "swiglu_epilogue", None))
        st = []
        for c in range(C):
            b0, b1 = bounds[c], bounds[c + 1]
            assert ((b1 - b0) * T) % n == 0, "sequence parallelism: chunk rows must divide by tp_size"
            ids_c = ids[b0:b1].reshape(-1).contiguous()
            x_s, h = _rs(k.embedding_fwd(ids_c, emb.weight, emb.vocab_st_idx, dt), n)
            # the embedding backward's sort, on a side stream beside the forward
            esort = emb_sort_ahead(ids_c, emb.vocab_st_idx, emb.weight.size(0)) if k is not reference else None
            st.append(dict(B=b1 - b0, ids=ids_c, esort=esort, pos=pos[b0:b1].reshape(-1).contiguous(),
                           tgt=tgt[b0:b1].reshape(-1).contiguous(), x=x_s, h=h, pend=None, pend_bias=None,
                           layers=[]))
        for L in layers:
            for s in st:    # P1: (bias + residual +) norm1 on my rows -> all-gather
                _wait(s["h"])
                if s["pend"] is not None:
                    s["x"], h1s, r1 = k.add_rmsnorm_fwd(s["pend"], s["pend_bias"], s["x"], L.s1, L.eps1)
                else:
                    h1s, r1 = k.rmsnorm_fwd(s["x"], L.s1, L.eps1)
                h1, s["h"] = _ag(h1s, n)
                s["layers"].append(dict(x=s["x"], r1=r1, h1=h1))
            for ci, s in enumerate(st):    # P2: QKV (+RoPE), attention, Wo -> reduce-scatter
                _wait(s["h"])
                a = s["layers"][-1]
                qkv = GS.gemm_nt_rope(k, a["h1"], W(L.wqkv), L.bqkv, s["pos"], tab, 2 * L.h, L.hd)
                q, kk, v = _split(qkv, s["B"], T, L.h, L.hd)
                o, lse = k.attn_fwd(q, kk, v, 1.0 / math.sqrt(L.hd), True)
                pout = GS.gemm_nt(k, o.view(qkv.size(0), L.h * L.hd), W(L.wo), None,
                                  out=_slot(ci, qkv.size(0), d, dt))
                a.update(qkv=qkv, o=o, lse=lse)
                (s["pend"], s["h"]), s["pend_bias"] = _rs(pout, n), L.bo
            for s in st:    # P3: bias + residual + norm2 on my rows -> all-gather
                _wait(s["h"])
                a = s["layers"][-1]
                x2, h2s, r2 = k.add_rmsnorm_fwd(s["pend"], s["pend_bias"], s["x"], L.s2, L.eps2)
                h2, s["h"] = _ag(h2s, n)
                a.update(x2=x2, r2=r2, h2=h2)
                s["x"] = x2
            for ci, s in enumerate(st):    # P4: gate|up, SwiGLU, down -> reduce-scatter
                _wait(s["h"])
                a = s["layers"][-1]
                gu, sw = GS.gate_up(k, a["h2"], W(L.wgu), L.bgu, L.swi)   # SwiGLU in the epilogue
                qout = GS.gemm_nt(k, sw, W(L.wd), None, out=_slot(ci, sw.size(0), d, dt))
                a.update(gu=gu, sw=sw)
                (s["pend"], s["h"]), s["pend_bias"] = _rs(qout, n), L.bd
                if recompute:          # keep only the layer input; the rest is rebuilt in backward
                    s["layers"][-1] = {"x": a["x"]}
        for s in st:        # final norm on my rows -> all-gather
            _wait(s["h"])
            xf, hfs, rf = k.add_rmsnorm_fwd(s["pend"], s["pend_bias"], s["x"], model.norm.scale, model.norm.eps)
            hf, s["h"] = _ag(hfs, n)
            s.update(xf=xf, rf=rf, hf=hf)
            del s["pend"]
        acc = torch.empty(2, device=dev, dtype=torch.float32)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        for ci, s in enumerate(st):        # lm_head shard + vocab-parallel CE statistics
            _wait(s["h"])
            logits = GS.gemm_nt(k, s["hf"], W(head.weight), head.bias)
            stats = k.ce_fwd_stats(logits, s["tgt"], vst, vvalid)
            allst = stats.new_empty((n * stats.size(0), 3))
            dist.all_gather_into_tensor(allst, stats, group=p.tp_group)
            allst = allst.view(n, -1, 3)
            lse, valid = k.ce_finalize(allst, s["tgt"], ignore_index, acc, loss, ci == 0, ci == len(st) - 1)
            s.update(logits=logits, ce_lse=lse, valid=valid, h=None)
        ctx.model, ctx.st, ctx.layers, ctx.meta = model, st, layers, (T, dt, vst, vvalid, n)
        ctx.recompute = recompute
        ctx.n_valid, ctx.tab = acc[1], tab
        ctx.f8map = f8map
        F8.activate(None)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        model, st, layers = ctx.model, ctx.st, ctx.layers
        T, dt, vst, vvalid, n = ctx.meta
        k = K(model.embedding.weight, model.act_dtype(model.embedding.weight.device))
        head = model.lm_head
        W = lambda w: shadow(w, dt) if w is not None else None
        F8.activate(ctx.f8map)
        _defer_begin()
        tab = ctx.tab
        nL = len(layers)
        # fp32 gradients straight into the model's gradient arena (parallel/grad_sync.GradArena):
        # DP all-reduces run on contiguous slices of it, no pack / copy back
        arena = GSY.arena_for(model, arena_groups(model, layers, True), "sp")
        assign = arena_begin(model, arena)
        g = {"emb": None, "nf": None, "lm_w": None, "lm_b": None}
        gl = [dict() for _ in range(nL)]
        gname = {id(gl[li]): f"L{li}" for li in range(nL)}
        V = lambda d_, key: arena.view(gname.get(id(d_)) or ("tail" if key in ("emb", "nf") else "head"), key)

        def first(d_, key, like, n):
            """fp32 output buffer of a gradient kernel: the arena slot for the first chunk."""
            return V(d_, key) if d_.get(key) is None else like.new_empty(n, dtype=torch.float32)

        def tn(d, key, dy, x):
            if d.get(key) is None:
                d[key] = GS.gemm_tn(k, dy, x, V(d, key))
            else:
                GS.gemm_tn(k, dy, x, d[key], True)

        def tn_chunks(d, key, pairs):
            """Weight gradient summed over the chunks ((dy, x) per chunk), issued after the
            last chunk's data-gradient GEMM of the phase: chunks go two at a time through
            GS.gemm_tn_pair (one split-K launch over both chunks' rows, one reduction)."""
            i = 0
            while i < len(pairs):
                if i + 1 < len(pairs):
                    (a0, b0), (a1, b1) = pairs[i], pairs[i + 1]
                    if d.get(key) is None:
                        d[key] = GS.gemm_tn_pair(k, a0, b0, a1, b1, V(d, key), False)
                    else:
                        GS.gemm_tn_pair(k, a0, b0, a1, b1, d[key], True)
                    i += 2
                else:
                    tn(d, key, *pairs[i])
                    i += 1
            pairs.clear()

        def tn_multi(d, groups):
            """A phase's weight gradients ((key, pairs) each): with one or two chunks ONE grouped
            launch (GS.gemm_tn_group, timed against separate calls), else per key."""
            if all(len(pairs) == 1 for _, pairs in groups) or all(len(pairs) == 2 for _, pairs in groups):
                # (two chunks: each item's rows continue in the other chunk's buffers)
                items = []
                for key, pairs in groups:
                    acc = d.get(key)
                    items.append((pairs[0][0], pairs[0][1], acc if acc is not None else V(d, key), acc is not None)
                                 + (tuple(pairs[1]) if len(pairs) == 2 else ()))
                for (key, pairs), o in zip(groups, GS.gemm_tn_group(k, items)):
                    d[key] = o
                    pairs.clear()
                return
            for key, pairs in groups:
                tn_chunks(d, key, pairs)

        pg = pm.pgm
        dp = pg.dp_size
        # buckets of at least the measured knee of the DP group's all-reduce curve
        # (parallel/grad_sync.dp_bucket_bytes; small per-layer groups are merged)
        dpb = GSY.DPBucketer(arena, pg.dp_group if dp > 1 else None, dp,
                             GSY.dp_bucket_bytes(pg.dp_group, gloss.device) if dp > 1 else 0,
                             before_launch=_defer_flush)
        dp_reduce = dpb.add

        d = model.args.attn_dim
        lm_p = []
        for ci, s in enumerate(st):    # CE backward in place, lm_head dgrad -> reduce-scatter, lm_head wgrad
            gs = k.ce_grad_scale(s["valid"], gloss, ctx.n_valid)
            dl = s["logits"]
            db = first(g, "lm_b", dl, dl.size(1)) if head.bias is not None else None
            k.ce_bwd(dl, s["tgt"], s["ce_lse"], gs, vst, vvalid, dl, db)
            s["dpend"], s["h"] = _rs(GS.gemm_nn(k, dl, W(head.weight), out=_slot(ci, dl.size(0), d, dt)), n)
            lm_p.append((dl, s["hf"]))
            if db is not None:
                g["lm_b"] = _addg(g["lm_b"], db, V(g, "lm_b"))
            del s["logits"], s["hf"]
        tn_chunks(g, "lm_w", lm_p)
        def norm_bwd(dy, x, w, r, dres, bias_below, below_key):
            """RMSNorm backward on my rows (+ residual grad); the bias grad of the projection
            whose output feeds this residual (column sums of the result) from the same pass."""
            db = first(below_key[0], below_key[1], dy, dy.size(1)) if bias_below is not None else None
            out, ds = k.rmsnorm_bwd(dy, x, w, r, dres, db)
            if db is not None:
                below_key[0][below_key[1]] = _addg(below_key[0].get(below_key[1]), db, V(*below_key))
            return out, ds

        for s in st:    # final norm backward on my rows -> all-gather the residual grad
            _wait(s["h"])
            s["g"], dsf = norm_bwd(s["dpend"], s["xf"], model.norm.scale, s["rf"], None,
                                   layers[-1].bd, (gl[nL - 1], "bd"))
            g["nf"] = _addg(g["nf"], dsf, V(g, "nf"))
            s["gfull"], s["h"] = _ag(s["g"], n)
            del s["xf"], s["rf"], s["dpend"]
        dp_reduce("head")

        def rebuild(L, li):
            """Activation recompute: re-run layer li's forward (with its collectives) from the
            saved layer input, up to the SwiGLU output (the down projection is not needed)."""
            for s in st:
                a = s["layers"][li]
                h1s, a["r1"] = k.rmsnorm_fwd(a["x"], L.s1, L.eps1)
                a["h1"], a["hh"] = _ag(h1s, n)
            for ci, s in enumerate(st):
                a = s["layers"][li]
                _wait(a.pop("hh"))
                a["qkv"] = GS.gemm_nt_rope(k, a["h1"], W(L.wqkv), L.bqkv, s["pos"], tab, 2 * L.h, L.hd)
                q, kk, v = _split(a["qkv"], s["B"], T, L.h, L.hd)
                a["o"], a["lse"] = k.attn_fwd(q, kk, v, 1.0 / math.sqrt(L.hd), True)
                pout = GS.gemm_nt(k, a["o"].view(a["qkv"].size(0), L.h * L.hd), W(L.wo), None,
                                  out=_slot(ci, a["qkv"].size(0), d, dt))
                a["pend"], a["hh"] = _rs(pout, n)
            for s in st:
                a = s["layers"][li]
                _wait(a.pop("hh"))
                a["x2"], h2s, a["r2"] = k.add_rmsnorm_fwd(a.pop("pend"), L.bo, a["x"], L.s2, L.eps2)
                a["h2"], a["hh"] = _ag(h2s, n)
            for s in st:
                a = s["layers"][li]
                _wait(a.pop("hh"))
                a["gu"], a["sw"] = GS.gate_up(k, a["h2"], W(L.wgu), L.bgu, L.swi)

        for li in range(nL - 1, -1, -1):
            L, G = layers[li], gl[li]
            if ctx.recompute:
                rebuild(L, li)
            wd_p, wgu_p = [], []
            for ci, s in enumerate(st):    # B4: down / SwiGLU / gate|up grads -> reduce-scatter
                _wait(s["h"])
                a, gq = s["layers"][li], s["gfull"]
                # (bd's grad, partial over my rows and summed over TP by TrainStep, came out of
                # the norm backward above this layer)
                wd_p.append((gq, a["sw"]))
                dbgu = first(G, "bgu", gq, a["gu"].size(1)) if L.bgu is not None else None
                # down dgrad with the SwiGLU backward (+ gate|up bias grad) in its epilogue
                dgu = GS.down_dgrad_swiglu(k, gq, W(L.wd), a["gu"], dbgu, L.swi)
                s["dpend"], s["h"] = _rs(GS.gemm_nn(k, dgu, W(L.wgu), out=_slot(ci, dgu.size(0), d, dt)), n)
                wgu_p.append((dgu, a["h2"]))
                if dbgu is not None:
                    G["bgu"] = _addg(G.get("bgu"), dbgu, V(G, "bgu"))
                del a["sw"], a["gu"], a["h2"], s["gfull"]
            tn_multi(G, [("wd", wd_p), ("wgu", wgu_p)])       # under the chunks' reduce-scatters
            for s in st:    # B3: norm2 backward (+ residual grad) on my rows -> all-gather
                _wait(s["h"])
                a = s["layers"][li]
                s["g"], ds2 = norm_bwd(s["dpend"], a["x2"], L.s2, a["r2"], s["g"], L.bo, (G, "bo"))
                G["s2"] = _addg(G.get("s2"), ds2, V(G, "s2"))
                s["gfull"], s["h"] = _ag(s["g"], n)
                del a["x2"], a["r2"], s["dpend"]
            wo_p, wqkv_p = [], []
            for ci, s in enumerate(st):    # B2: Wo / attention / QKV grads -> reduce-scatter
                _wait(s["h"])
                a, g2 = s["layers"][li], s["gfull"]
                do = GS.gemm_nn(k, g2, W(L.wo))
                wo_p.append((g2, a["o"].view(g2.size(0), -1)))
                Bc = s["B"]
                q, kk, v = _split(a["qkv"], Bc, T, L.h, L.hd)
                dqkv = torch.empty_like(a["qkv"])
                dq, dk, dv = _split(dqkv, Bc, T, L.h, L.hd)
                dbq = first(G, "bqkv", dqkv, dqkv.size(1)) if L.bqkv is not None else None
                bq_fused = k.attn_bwd(do.view(Bc, T, L.h, L.hd), q, kk, v, a["o"], a["lse"], 1.0 / math.sqrt(L.hd),
                                      True, dq, dk, dv, s["pos"], tab, dbias=dbq)
                s["dpend"], s["h"] = _rs(GS.gemm_nn(k, dqkv, W(L.wqkv), out=_slot(ci, dqkv.size(0), d, dt)), n)
                wqkv_p.append((dqkv, a["h1"]))
                if L.bqkv is not None:
                    G["bqkv"] = _addg(G.get("bqkv"), dbq if bq_fused else k.bias_grad(dqkv), V(G, "bqkv"))
                for key in ("qkv", "o", "lse", "h1"):
                    a.pop(key, None)
                del s["gfull"]
            tn_multi(G, [("wo", wo_p), ("wqkv", wqkv_p)])
            for s in st:    # B1: norm1 backward (+ residual grad) on my rows -> all-gather
                _wait(s["h"])
                a = s["layers"][li]
                s["g"], ds1 = norm_bwd(s["dpend"], a["x"], L.s1, a["r1"], s["g"],
                                       layers[li - 1].bd if li > 0 else None, (gl[li - 1], "bd"))
                G["s1"] = _addg(G.get("s1"), ds1, V(G, "s1"))
                s["gfull"], s["h"] = _ag(s["g"], n)
                del a["x"], a["r1"], s["dpend"]
            dp_reduce(f"L{li}")
        ev = arena.view("tail", "emb")
        for ci, s in enumerate(st):    # embedding backward over all rows of the chunk (vocab-sharded table)
            _wait(s["h"])
            # deterministic (sorted ids, no atomics): chunk 0 writes every row, the rest add
            perm, seg = emb_sort_take(s.pop("esort", None))
            k.embedding_bwd_sorted(s["gfull"], s["ids"], model.embedding.weight.size(0),
                                   model.embedding.vocab_st_idx, out=ev, accumulate=ci > 0, perm=perm, seg=seg)
            del s["gfull"]
        g["emb"] = ev
        dp_reduce("tail")
        dp_reduce("sprep")
        _defer_end()
        tp_comm.check()
        if dpb.finish():
            model._dpfs_dp_reduced = True   # DataParallelGradSync hooks skip this step
        ctx.st = None
        grads = [g["emb"]]
        for li, L in enumerate(layers):
            G = gl[li]
            grads += [G["s1"], G["wqkv"], G.get("bqkv") if L.bqkv is not None else None,
                      G["wo"], G.get("bo") if L.bo is not None else None, G["s2"], G["wgu"],
                      G.get("bgu") if L.bgu is not None else None, G["wd"],
                      G.get("bd") if L.bd is not None else None]
        grads += [g["nf"], g["lm_w"], g["lm_b"] if head.bias is not None else None]
        F8.activate(None)
        return (None, None, None, None, None, None) + tuple(arena_end(model, grads, assign))
