"""Per-rank HBM planner for the explicit-schedule training step (288 GB per MI355X).

The reference sizes nothing: it logs ``torch.cuda.memory_reserved`` after the fact
(``train.py:119-120``) and a run that does not fit dies with an allocator error.  Here every
tensor the fused engines (``models/fused_engine.py``, ``models/fused_engine_sp.py``) keep
alive is counted before the model is built, per rank, for a given layout
(preset x TP x DP x SP x seq x batch x ping-pong chunks x recompute):

* static state -- fp32 master weights, the bf16 compute shadows of the 2-D weights (written by
  the fused Adam), Adam's two fp32 moments, and the fp32 gradient arena
  (``parallel/grad_sync.GradArena``: one buffer for every gradient of the step, written in
  place by the backward, so the previous step's gradients never coexist with this step's);
* activations saved per layer and chunk (x, normed inputs, roped QKV, attention output + LSE,
  gate|up, SwiGLU output; under SP the residual stream and norms on 1/TP of the rows; with
  recompute only each layer's input, plus one rebuilt layer in backward);
* the head: final norm outputs and the bf16 logits shard, which the vocab-parallel CE keeps
  until the backward (its gradient is written in place);
* the backward's largest transient: the lm_head weight gradient with its split-K slabs, or
  one layer's data / weight-gradient temporaries;
* the xGMI staging buffers of the TP collectives.

``plan`` compares the peak with the device's free bytes (``torch.cuda.mem_get_info``) minus a
margin, turns recompute on when only that fits, and refuses a layout that does not fit at all,
with the numbers in the error.  ``tests/test_memory_plan.py`` covers the arithmetic on the CPU;
``tests/test_memory_gpu.py`` checks the estimate against ``torch.cuda.max_memory_allocated``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

from ..models.config import ModelArgs, vocab_partition
from ..parallel.layers import partition_sizes

GiB = float(1 << 30)


@dataclass
class Layout:
    tp: int = 1
    dp: int = 1
    sp: bool = False
    seq: int = 1024
    batch: int = 32            # sequences per DP replica (= per TP group) per step
    chunks: int = 1            # ping-pong chunks of the fused engine
    recompute: bool = False
    tp_rank: int = 0           # the rank to size (uneven head / vocab shards: use the largest)
    compute: str = "bf16"      # "bf16" | "fp32": activation bytes; fp32 keeps no bf16 shadows
    materialized_attention: bool = False   # the PyTorch oracle path: (B, H, T, T) fp32 scores


def xgmi_staging_bytes(tp: int, cap_mb: Optional[int] = None, nslots: int = 4) -> int:
    """Bytes ``csrc/comm/xgmi.hip`` ``dpfs_xgmi_create`` allocates per rank: nslots staging
    slots + the copy-in and temporary regions (nslots + 2 capacities) + two one-shot input
    regions of min(capacity, 16 MiB); the capacity is ``DPFS_XGMI_CAP_MB`` (256 default)."""
    if tp <= 1:
        return 0
    import os
    cap = (cap_mb if cap_mb is not None else int(os.environ.get("DPFS_XGMI_CAP_MB", "256"))) << 20
    return (nslots + 2) * cap + 2 * min(cap, 16 << 20)


@dataclass
class Estimate:
    parts: Dict[str, int] = field(default_factory=dict)   # bytes
    peak: int = 0
    phase: str = ""            # "forward" | "backward": where the peak is

    def gb(self) -> float:
        return self.peak / GiB

    def table(self) -> str:
        rows = [f"{k:>22}: {v / GiB:8.2f} GiB" for k, v in self.parts.items()]
        return "\n".join(rows + [f"{'peak (' + self.phase + ')':>22}: {self.peak / GiB:8.2f} GiB"])


def _tn_splits(M: int, N: int, K: int) -> int:
    """K-splits of the fp32 weight-gradient GEMM (csrc/kernels/gemm.hip tn_v2_splits, the
    makespan model over 256 CUs): the slab workspace is splits x M x N fp32."""
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    best, best_t = 1, 1e300
    for S in range(1, 65):
        if S > 1 and K // S < 512:
            break
        kps = ((K + S - 1) // S + 63) // 64
        rounds = (tiles * S + 255) // 256
        t = rounds * kps * 1.95 + (S * M * N * 8.0 / 4.0e6 if S > 1 else 0.0)
        if t < best_t * 0.97:
            best_t, best = t, S
    return best


def estimate(args: ModelArgs, lay: Layout, act_bytes: Optional[int] = None) -> Estimate:
    """Peak bytes allocated on one rank during a steady-state training step.  ``act_bytes``
    defaults from ``lay.compute`` (2 for bf16, 4 for fp32)."""
    if act_bytes is None:
        act_bytes = 4 if lay.compute == "fp32" else 2
    n, r = lay.tp, min(lay.tp_rank, lay.tp - 1)
    d, F, L, hd = args.attn_dim, args.ffn_dim, args.num_layers, args.head_dim
    dl = partition_sizes(d, n, hd)[r]                  # this rank's attention width (heads x hd)
    Fl = partition_sizes(F, n)[r]
    heads = [w // hd for w in partition_sizes(d, n, hd)]
    Vl = vocab_partition(args, heads)[r]
    b = 1 if args.bias else 0
    # ---- parameters on this rank (sharded + replicated)
    w2d_layer = 3 * dl * d + d * dl + 2 * Fl * d + d * Fl
    p_layer = w2d_layer + b * (3 * dl + d + 2 * Fl + d) + 2 * d * (2 if args.norm == "layernorm" else 1)
    w2d = L * w2d_layer + 2 * Vl * d                   # + embedding and lm_head shards
    P = L * p_layer + 2 * Vl * d + b * Vl + d * (2 if args.norm == "layernorm" else 1)
    parts: Dict[str, int] = {}
    parts["master_fp32"] = 4 * P
    parts["shadow_bf16"] = 2 * w2d if lay.compute != "fp32" else 0
    parts["adam_m_v_fp32"] = 8 * P
    parts["grad_arena_fp32"] = 4 * P
    static = parts["master_fp32"] + parts["shadow_bf16"] + parts["adam_m_v_fp32"] + parts["grad_arena_fp32"]

    # ---- activations: M = tokens per TP group per step, over all chunks
    M = lay.batch * lay.seq
    a = act_bytes
    rows_sp = M // n if lay.sp else M                   # rows of the residual stream / norms
    per_layer = (a * rows_sp * d * 2                    # x, x2 (residual stream)
                 + 4 * rows_sp * 2                      # r1, r2 (fp32 rstd)
                 + a * M * d * 2                        # h1, h2 (normed inputs, full rows)
                 + a * M * 3 * dl                       # roped QKV
                 + a * M * dl                           # attention output
                 + 4 * M * (dl // hd)                   # log-sum-exp (fp32 per head and row)
                 + a * M * 3 * Fl)                      # gate|up + SwiGLU output
    layer_in = a * rows_sp * d
    acts = L * (layer_in if lay.recompute else per_layer)
    parts["activations"] = acts
    # xf (residual rows), rf, hf (normed, full rows), the logits shard, CE lse / validity
    head = a * rows_sp * d + 4 * rows_sp + a * M * d + a * M * Vl + 4 * M * 3
    parts["head_logits_etc"] = head
    # ---- backward transients beside the live activations
    sl = _tn_splits(Vl, d, M)
    lm_tn = 4 * Vl * d * (1 + (sl if sl > 1 else 0))   # lm_head weight grad + its split-K slabs
    layer_tmp = a * M * (3 * dl + 2 * Fl + 2 * d) + 4 * max(
        _tn_splits(2 * Fl, d, M) * 2 * Fl * d, _tn_splits(3 * dl, d, M) * 3 * dl * d,
        _tn_splits(d, Fl, M) * d * Fl, _tn_splits(d, dl, M) * d * dl)
    rebuilt = per_layer if lay.recompute else 0
    if lay.materialized_attention:
        # the oracle keeps every layer's (tokens x T) fp32 probabilities for its backward, and
        # one layer's scores + probabilities + their gradient transiently
        heads_l = dl // hd
        scores = 4 * M * lay.seq * heads_l
        parts["attention_scores"] = L * scores
        acts += L * scores
        layer_tmp += 2 * scores
    parts["bwd_transient"] = max(lm_tn + a * M * d, layer_tmp + rebuilt)
    parts["xgmi_staging"] = xgmi_staging_bytes(n)
    fwd_peak = static + acts + head + parts["xgmi_staging"]
    bwd_peak = static + acts + head + parts["bwd_transient"] + parts["xgmi_staging"]
    est = Estimate(parts=parts)
    est.peak, est.phase = (fwd_peak, "forward") if fwd_peak >= bwd_peak else (bwd_peak, "backward")
    return est


class DoesNotFit(MemoryError):
    pass


def plan(args: ModelArgs, lay: Layout, free_bytes: Optional[int] = None, recompute: Optional[bool] = None,
         margin_frac: float = 0.06, margin_bytes: int = 2 << 30):
    """(recompute, estimate): ``recompute`` None = decide (off if the layout fits without it,
    else on if that fits); True / False = the caller's choice, checked.  Raises ``DoesNotFit``
    (with the per-part table) when the chosen layout exceeds ``free_bytes`` minus the margin.
    ``free_bytes`` None: no budget (the estimate is returned, nothing is refused)."""
    budget = None if free_bytes is None else int(free_bytes * (1 - margin_frac)) - margin_bytes
    e0 = estimate(args, Layout(**{**lay.__dict__, "recompute": False}))
    e1 = estimate(args, Layout(**{**lay.__dict__, "recompute": True}))
    if recompute is None:
        if budget is None or e0.peak <= budget:
            return False, e0
        recompute = True
    e = e1 if recompute else e0
    if budget is not None and e.peak > budget:
        alt = "" if recompute else f"; with recompute {e1.gb():.1f} GiB"
        raise DoesNotFit(f"layout tp{lay.tp} dp{lay.dp}{' sp' if lay.sp else ''} seq {lay.seq} batch {lay.batch} "
                         f"chunks {lay.chunks} recompute={recompute}: estimated peak {e.gb():.1f} GiB per rank > "
                         f"budget {budget / GiB:.1f} GiB (free {free_bytes / GiB:.1f} GiB){alt}\n{e.table()}")
    return recompute, e


def device_free_bytes(device=None) -> Optional[int]:
    """Free bytes of the current (or given) GPU; None without one."""
    import torch
    if not torch.cuda.is_available():
        return None
    free, _total = torch.cuda.mem_get_info(device)
    return int(free)
