"""Pure-PyTorch reference kernels: the CPU compute path and the numerical oracle.

Every function here has the *same signature and semantics* as the HIP kernel of the same
name in ``csrc/kernels`` (exported by ``_C``).  Tests compare the two; on CPU the model runs
on these.  Math is done in fp32 and results are cast to the input dtype, matching the GPU
kernels' accumulate-in-fp32 policy.

Reference parity notes (``/root/reference``):

* ``rmsnorm_fwd``: ``models/layers.py:145-155`` (``scale * (x * rsqrt(mean(x^2)+eps))``).
* ``rope_``: ``models/model.py:17-46`` (HF rotate-half; cos/sin tables with duplicated
  halves, angles ``pos * theta`` in fp32).
* ``attention``: ``models/model.py:73-77`` (causal, softmax(QK^T/sqrt(hd)) V).
* ``swiglu``: ``models/model.py:94-95``.
* ``embedding_fwd``: ``models/layers.py:134-141`` without the in-place mutation of the ids.
* ``vocab-parallel CE``: extension; the reference all-gathers logits and calls
  ``F.cross_entropy(ignore_index=-1)`` (``train.py:101-104``).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


# ------------------------------------------------------------------------------- GEMM ----

def gemm_nt(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None, rope_pos=None, rope_tab=None,
            rope_heads: int = 0, rope_hd: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """c[M,N] = a[M,K] @ b[N,K]^T (+ bias[N]); output dtype = a.dtype.  With ``rope_pos`` the first
    ``rope_heads`` heads of each row are then rotated (the GPU kernel fuses this into its
    epilogue)."""
    c = a.float() @ b.float().t()
    if bias is not None:
        c = c + bias.float()
    c = c.to(a.dtype)
    if rope_pos is not None and rope_heads > 0:
        rope_(c, rope_pos, rope_tab, rope_heads, rope_hd, False)
    return out.copy_(c) if out is not None else c


def gemm_nn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """c[M,N] = a[M,K] @ b[K,N]; output dtype = a.dtype (written into ``out`` when given)."""
    c = (a.float() @ b.float()).to(a.dtype)
    return out.copy_(c) if out is not None else c


def gemm_tn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
            accumulate: bool = False) -> torch.Tensor:
    """c[M,N] (fp32) = a[K,M]^T @ b[K,N]  (+= into ``out`` if ``accumulate``)."""
    c = a.float().t() @ b.float()
    if out is None:
        return c
    if accumulate:
        out.add_(c)
    else:
        out.copy_(c)
    return out


def gemm_tn2(a0: torch.Tensor, b0: torch.Tensor, a1: torch.Tensor, b1: torch.Tensor,
             out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """c[M,N] (fp32) = a0^T b0 + a1^T b1: a TN GEMM whose reduction dim is split over two
    buffers (+= into ``out`` if ``accumulate``)."""
    c = gemm_tn(a0, b0, out, accumulate)
    return gemm_tn(a1, b1, c, True)


def add_bias_(y: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """y[M,N] += bias[N] in place (fp32 add, rounded to y.dtype); returns y."""
    y.copy_((y.float() + bias.float()).to(y.dtype))
    return y


def bias_residual(y: torch.Tensor, bias: Optional[torch.Tensor], residual: torch.Tensor) -> torch.Tensor:
    """out = residual + y (+ bias), fp32 math, rounded once to y.dtype."""
    out = y.float() + residual.float()
    if bias is not None:
        out = out + bias.float()
    return out.to(y.dtype)


def bias_grad(dy: torch.Tensor) -> torch.Tensor:
    """fp32 column sums of dy[M,N]."""
    return dy.float().sum(0)


# -------------------------------------------------------------------------- norms ----

def rmsnorm_fwd(x: torch.Tensor, w: torch.Tensor, eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1) + eps)
    y = (xf * rstd[:, None]).to(x.dtype).float() * w.float()
    return y.to(x.dtype), rstd


def rmsnorm_bwd(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, rstd: torch.Tensor,
                dres: Optional[torch.Tensor] = None, dbias: Optional[torch.Tensor] = None,
                dw_out: Optional[torch.Tensor] = None):
    """Returns (dx [+ dres if given, fused residual-grad add], dw fp32); with ``dbias`` (fp32
    [D]) also writes the column sums of dx there (the bias grad of the layer below); with
    ``dw_out`` (fp32 [D]) dw is written there and returned."""
    xf, dyf, wf = x.float(), dy.float(), w.float()
    xhat = xf * rstd[:, None]
    dw = (dyf * xhat).sum(0)
    g = dyf * wf
    d = xf.size(-1)
    dx = rstd[:, None] * (g - xhat * (g * xhat).sum(-1, keepdim=True) / d)
    if dres is not None:
        dx = dx + dres.float()
    if dbias is not None:
        dbias.copy_(dx.sum(0))
    if dw_out is not None:
        dw = dw_out.copy_(dw)
    return dx.to(x.dtype), dw


def add_rmsnorm_fwd(y: torch.Tensor, bias: Optional[torch.Tensor], res: torch.Tensor, w: torch.Tensor,
                    eps: float):
    """(x = y + bias + res rounded to y.dtype, rmsnorm_fwd(x)) — the fused residual epilogue."""
    x = bias_residual(y, bias, res)
    h, rstd = rmsnorm_fwd(x, w, eps)
    return x, h, rstd


def layernorm_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float):
    xf = x.float()
    mean = xf.mean(-1)
    var = (xf - mean[:, None]).pow(2).mean(-1)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mean[:, None]) * rstd[:, None] * w.float() + b.float()
    return y.to(x.dtype), mean, rstd


def layernorm_bwd(dy, x, w, mean, rstd):
    xf, dyf, wf = x.float(), dy.float(), w.float()
    xhat = (xf - mean[:, None]) * rstd[:, None]
    dw = (dyf * xhat).sum(0)
    db = dyf.sum(0)
    g = dyf * wf
    d = xf.size(-1)
    dx = rstd[:, None] * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).sum(-1, keepdim=True) / d)
    return dx.to(x.dtype), dw, db


# --------------------------------------------------------------------------- RoPE ----

def rope_table(maxlen: int, head_dim: int, theta: float, device=None) -> torch.Tensor:
    """fp32 ``(maxlen, head_dim)`` table: columns [cos(pos*inv_freq) | sin(pos*inv_freq)] for
    the ``head_dim/2`` frequencies (the reference duplicates each half; we store it once).
    ``inv_freq`` is computed on CPU in fp32 exactly as ``models/model.py:38``."""
    assert head_dim % 2 == 0
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    pos = torch.arange(maxlen).float().unsqueeze(1)
    ang = pos * inv
    tab = torch.cat([torch.cos(ang), torch.sin(ang)], dim=1)
    return tab.to(device) if device is not None else tab


def rope_(qkv: torch.Tensor, positions: torch.Tensor, table: torch.Tensor, n_rot_heads: int,
          head_dim: int, inverse: bool = False) -> torch.Tensor:
    """Rotate (in place) the first ``n_rot_heads`` heads of each row of ``qkv[M, *]``.

    ``positions[M]`` indexes ``table``.  ``inverse`` applies the transpose rotation (the RoPE
    backward).  Rotate-half convention: out1 = x1 c - x2 s, out2 = x2 c + x1 s.
    """
    M = qkv.size(0)
    h2 = head_dim // 2
    tab = table[positions.long()]  # (M, hd)
    c = tab[:, None, :h2]
    s = tab[:, None, h2:]
    if inverse:
        s = -s
    view = qkv[:, : n_rot_heads * head_dim].view(M, n_rot_heads, head_dim)
    x1 = view[..., :h2].float()
    x2 = view[..., h2:].float()
    o1 = x1 * c - x2 * s
    o2 = x2 * c + x1 * s
    view[..., :h2] = o1.to(qkv.dtype)
    view[..., h2:] = o2.to(qkv.dtype)
    return qkv


# ---------------------------------------------------------------------- attention ----

def attn_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float,
             causal: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """q,k,v: (B, T, H, hd) (any strides). Returns o (B, T, H, hd) contiguous and the
    natural-log LSE (B, H, T) fp32 of the scaled scores."""
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))  # B H T hd
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        T, S = s.shape[-2], s.shape[-1]
        mask = torch.ones(T, S, dtype=torch.bool, device=s.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse[..., None])
    o = (p @ vf).transpose(1, 2).contiguous()
    return o.to(q.dtype), lse


def attn_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, len: torch.Tensor,
                scale: float) -> torch.Tensor:
    """One query row per (sequence, head) against cache rows [0, len]: q [B, >= H*hd] rows,
    caches (B, T_max, H, hd), len a 1-element int tensor.  Returns o [B, H*hd] in q.dtype."""
    B, _, H, hd = k_cache.shape
    L = int(len.reshape(-1)[0]) + 1
    qf = q[:, : H * hd].float().view(B, H, 1, hd)
    kf = k_cache[:, :L].float().transpose(1, 2)          # B H L hd
    vf = v_cache[:, :L].float().transpose(1, 2)
    p = torch.softmax((qf @ kf.transpose(-1, -2)) * scale, dim=-1)
    return (p @ vf).reshape(B, H * hd).to(q.dtype)


def kv_append(qkv: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, len: torch.Tensor) -> None:
    """cache[:, len] = the k / v parts of the packed qkv rows [B, 3*H*hd]."""
    B, _, H, hd = k_cache.shape
    t = int(len.reshape(-1)[0])
    k_cache[:, t] = qkv[:, H * hd: 2 * H * hd].view(B, H, hd).to(k_cache.dtype)
    v_cache[:, t] = qkv[:, 2 * H * hd: 3 * H * hd].view(B, H, hd).to(v_cache.dtype)


def gemv_nt_ok(x: torch.Tensor, w: torch.Tensor, swiglu: bool = False) -> bool:
    return True


def gemv_nt(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
            swiglu: bool = False) -> torch.Tensor:
    """y = a w^T (+ bias) in x.dtype, a = x, or with ``swiglu`` a = silu(g) * u of the packed
    x = [g | u] rounded to x.dtype (the GPU kernel's fused operand; swiglu_fwd's rounding)."""
    if swiglu:
        K = w.size(1)
        g, u = x[:, :K].float(), x[:, K:].float()
        a = (g / (1.0 + torch.exp(-g)) * u).to(x.dtype)
    else:
        a = x
    y = a.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    return y.to(x.dtype)


def rope_append(qkv: torch.Tensor, pos: torch.Tensor, table: torch.Tensor, k_cache: torch.Tensor,
                v_cache: torch.Tensor, len: torch.Tensor) -> None:
    """rope_ on the q and k heads of the packed rows, then kv_append (one GPU kernel)."""
    H, hd = k_cache.size(2), k_cache.size(3)
    rope_(qkv, pos, table, 2 * H, hd, False)
    kv_append(qkv, k_cache, v_cache, len)


def step_advance(len: torch.Tensor, pos: torch.Tensor) -> None:
    len += 1
    pos.fill_(int(len.reshape(-1)[0]))


def _rot_bthd(x: torch.Tensor, positions: torch.Tensor, table: torch.Tensor, inverse: bool) -> torch.Tensor:
    """Rotate-half RoPE of an fp32 (B, T, H, hd) tensor; ``positions`` is flat [B*T]."""
    B, T, H, hd = x.shape
    h2 = hd // 2
    tab = table[positions.long()].view(B, T, 1, hd)
    c, s = tab[..., :h2], tab[..., h2:]
    if inverse:
        s = -s
    x1, x2 = x[..., :h2], x[..., h2:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def attn_bwd(do, q, k, v, o, lse, scale: float, causal: bool, dq_out, dk_out, dv_out, rope_pos=None,
             rope_tab=None, dbias=None):
    """Writes dq/dk/dv into the given (B, T, H, hd) views (packed dqkv buffer).  With
    ``rope_pos`` the inverse RoPE is applied to dq and dk (fused into the stores on the GPU).
    With ``dbias`` (fp32 [3 * H * hd]) also the packed QKV bias gradient: the column sums of
    dq | dk | dv over all tokens.  Returns whether ``dbias`` was written."""
    qf, kf, vf, dof, of = (t.float().transpose(1, 2) for t in (q, k, v, do, o))
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        T, S = s.shape[-2], s.shape[-1]
        mask = torch.ones(T, S, dtype=torch.bool, device=s.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.exp(s - lse[..., None])
    dv = p.transpose(-1, -2) @ dof
    dp = dof @ vf.transpose(-1, -2)
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = ds @ kf
    dk = ds.transpose(-1, -2) @ qf
    dq, dk = dq.transpose(1, 2), dk.transpose(1, 2)
    if rope_pos is not None:
        dq = _rot_bthd(dq, rope_pos, rope_tab, True)
        dk = _rot_bthd(dk, rope_pos, rope_tab, True)
    dq_out.copy_(dq)
    dk_out.copy_(dk)
    dv_out.copy_(dv.transpose(1, 2))
    if dbias is None:
        return False
    dbias.copy_(torch.cat([t.float().sum((0, 1)).reshape(-1) for t in (dq, dk, dv.transpose(1, 2))]))
    return True


# ------------------------------------------------------------------------- SwiGLU ----

def gu_perm(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """Interleave a packed [gate | up] dimension (size 2F, F % 64 == 0) in 64-blocks: positions
    [128 b, 128 b + 64) = gate [64 b, 64 b + 64), the next 64 = up [64 b, 64 b + 64).  The fused
    gate|up GEMM epilogue (csrc/kernels/gemm4.hip SwiOut) then holds each gate / up pair in one
    lane.  ``gu_unperm`` is the inverse."""
    n = x.size(dim)
    sh = list(x.shape)
    v = x.reshape(sh[:dim] + [2, n // 128, 64] + sh[dim + 1:])
    return v.transpose(dim, dim + 1).reshape(sh)


def gu_unperm(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
    n = x.size(dim)
    sh = list(x.shape)
    v = x.reshape(sh[:dim] + [n // 128, 2, 64] + sh[dim + 1:])
    return v.transpose(dim, dim + 1).reshape(sh)


def _gate_up(gu: torch.Tensor, perm: bool):
    if perm:
        gu = gu_unperm(gu, gu.dim() - 1)
    F_ = gu.size(-1) // 2
    return gu[..., :F_].float(), gu[..., F_:].float()


def swiglu_fwd(gu: torch.Tensor, perm: bool = False) -> torch.Tensor:
    """h = silu(gate) * up of a packed gate|up tensor (``perm``: interleaved, see gu_perm)."""
    g, u = _gate_up(gu, perm)
    return (F.silu(g) * u).to(gu.dtype)


def gemm_nt_swiglu(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None):
    """Gate|up projection with the SwiGLU of the fused GPU epilogue: b / bias in the natural
    [gate | up] layout, multiplied with the rows interleaved by gu_perm -> [gu (interleaved,
    a.dtype), h = silu(gate) * up (a.dtype)]."""
    gu = gemm_nt(a, gu_perm(b), gu_perm(bias) if bias is not None else None)
    return [gu, swiglu_fwd(gu, True)]


def swiglu_bwd(dh: torch.Tensor, gu: torch.Tensor, dbias: Optional[torch.Tensor] = None,
               perm: bool = False) -> torch.Tensor:
    """d gate|up in the natural [gate | up] layout (``perm``: gu is read interleaved); with
    ``dbias`` (fp32 [2F]) also writes the bias gradient (column sums)."""
    g, u = _gate_up(gu, perm)
    dhf = dh.float()
    sig = torch.sigmoid(g)
    silu = g * sig
    dg = dhf * u * sig * (1 + g * (1 - sig))
    du = dhf * silu
    d = torch.cat([dg, du], dim=-1)
    if dbias is not None:
        dbias.copy_(d.sum(0))
    return d.to(gu.dtype)


def gemm_nn_swiglu_bwd(dy: torch.Tensor, w: torch.Tensor, gu: torch.Tensor, dbias: Optional[torch.Tensor] = None,
                       perm: bool = True):
    """The down projection's data gradient fused with the SwiGLU backward (the GPU kernel's
    epilogue form): ds = dy w rounded to dy.dtype, then swiglu_bwd(ds, gu, dbias, perm).
    Returns [dgu]."""
    return [swiglu_bwd(gemm_nn(dy, w), gu, dbias, perm)]


# ---------------------------------------------------------------------- embedding ----

def embedding_fwd(ids: torch.Tensor, weight: torch.Tensor, vocab_start: int,
                  out_dtype: torch.dtype) -> torch.Tensor:
    """Rows of the local vocab shard for ids in [vocab_start, vocab_start+V_local), zeros
    elsewhere.  Does not mutate ``ids`` (the reference does, ``layers.py:138``)."""
    vl = weight.size(0)
    local = ids.long() - vocab_start
    m = (local >= 0) & (local < vl)
    out = weight[local.clamp(0, vl - 1)].float() * m[:, None].float()
    return out.to(out_dtype)


def embedding_bwd(dout: torch.Tensor, ids: torch.Tensor, v_local: int, vocab_start: int,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 dW[v_local, D] of the masked embedding (rows ADDED to ``out`` when given)."""
    local = ids.long() - vocab_start
    m = (local >= 0) & (local < v_local)
    dw = out if out is not None else torch.zeros(v_local, dout.size(-1), dtype=torch.float32, device=dout.device)
    dw.index_add_(0, local[m], dout[m].float())
    return dw


def embedding_bwd_sorted(dout: torch.Tensor, ids: torch.Tensor, v_local: int, vocab_start: int,
                         out: Optional[torch.Tensor] = None, accumulate: bool = False, perm=None,
                         seg=None) -> torch.Tensor:
    """``embedding_bwd`` that WRITES every row of ``out`` (``accumulate``: adds, as the later
    chunks of the engines), summing each vocab row's gradient rows in row order.  (``perm`` /
    ``seg``: the native kernel's precomputed sort, see ``emb_sort_ahead``; unused here.)"""
    if out is None:
        out = torch.zeros(v_local, dout.size(-1), dtype=torch.float32, device=dout.device)
    elif not accumulate:
        out.zero_()
    return embedding_bwd(dout, ids, v_local, vocab_start, out)


def emb_sort(ids: torch.Tensor, vocab_start: int, v_local: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(perm, seg): the ids' stable order by local vocab row with the ids outside the shard last,
    and each local row's segment start (seg[v_local] = number of in-shard ids)."""
    local = ids.reshape(-1).long() - vocab_start
    key = torch.where((local >= 0) & (local < v_local), local, torch.full_like(local, 0xFFFF))
    sk, perm = torch.sort(key, stable=True)
    seg = torch.searchsorted(sk, torch.arange(v_local + 1, device=ids.device))
    return perm, seg


def emb_sort_ahead(ids: torch.Tensor, vocab_start: int, v_local: int):
    """The embedding backward's sort (see ops.dispatch.emb_sort_ahead); nothing to do here."""
    return None


# ------------------------------------------------------------ vocab-parallel CE ----

def ce_fwd_stats(logits: torch.Tensor, targets: torch.Tensor, vocab_start: int,
                 vocab_valid: int) -> torch.Tensor:
    """Per-row local statistics of one vocab shard: (M, 3) fp32 = [max, sum(exp(x-max)),
    target_logit (0 if the target is not in this shard)].  Columns ``>= vocab_valid`` (the
    padded vocab tail inside this shard) are excluded."""
    x = logits.float()
    if vocab_valid < x.size(1):
        x = x[:, :vocab_valid]
    mx = x.max(dim=1).values
    se = torch.exp(x - mx[:, None]).sum(1)
    local = targets.long() - vocab_start
    hit = (local >= 0) & (local < x.size(1))
    tl = torch.where(hit, x.gather(1, local.clamp(0, max(x.size(1) - 1, 0))[:, None]).squeeze(1),
                     torch.zeros_like(mx))
    return torch.stack([mx, se, tl], dim=1)


def ce_combine(stats: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """stats: (n_shards, M, 3) gathered from every TP rank -> (lse[M], target_logit[M])."""
    mx = stats[..., 0].max(0).values
    se = (stats[..., 1] * torch.exp(stats[..., 0] - mx[None])).sum(0)
    lse = mx + torch.log(se)
    tl = stats[..., 2].sum(0)
    return lse, tl


def ce_finalize(stats: torch.Tensor, targets: torch.Tensor, ignore_index: int, acc: torch.Tensor,
                loss: torch.Tensor, first: bool, last: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """Loss bookkeeping from the gathered (n_shards, M, 3) statistics: returns (lse[M], valid[M]
    as 1.0 / 0.0); ``acc[0:2]`` holds the running (sum over valid rows of lse - target logit,
    valid count), overwritten when ``first``; with ``last`` the count is clamped to >= 1 and
    ``loss`` (0-d) gets the mean."""
    lse, tl = ce_combine(stats)
    valid = (targets != ignore_index).float()
    part = torch.stack([torch.where(valid > 0, lse - tl, torch.zeros_like(lse)).sum(), valid.sum()])
    if first:
        acc[:2] = part
    else:
        acc[:2] += part
    if last:
        acc[1] = acc[1].clamp_min(1.0)
        loss.copy_(acc[0] / acc[1])
    return lse, valid


def ce_valid_scale(targets: torch.Tensor, ignore_index: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(gs[M], n_valid): 1 / max(#valid, 1) on the valid rows, 0 on the ignored ones."""
    valid = (targets != ignore_index).float()
    n = valid.sum().clamp_min(1.0)
    return valid / n, n


def ce_grad_scale(valid: torch.Tensor, gloss: torch.Tensor, n_valid: torch.Tensor) -> torch.Tensor:
    """Per-row gradient scale of the CE backward: valid * gloss / n_valid."""
    return valid * (gloss.float().reshape(()) / n_valid.reshape(()))


def ce_bwd(logits: torch.Tensor, targets: torch.Tensor, lse: torch.Tensor, gscale: torch.Tensor,
           vocab_start: int, vocab_valid: int, out: torch.Tensor,
           dbias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """d logits = (softmax - onehot) * gscale[row] (gscale = 0 on ignored rows); padded
    columns get 0.  Written to ``out`` (may alias ``logits``: the GPU kernel runs in place)."""
    x = logits.float()
    p = torch.exp(x - lse[:, None])
    local = targets.long() - vocab_start
    hit = (local >= 0) & (local < vocab_valid)
    p[hit, local[hit]] -= 1.0
    p = p * gscale[:, None]
    if vocab_valid < x.size(1):
        p[:, vocab_valid:] = 0
    if dbias is not None:
        dbias.copy_(p.sum(0))
    out.copy_(p)
    return out


def ce_fused(logits: torch.Tensor, targets: torch.Tensor, gscale: torch.Tensor, vocab_start: int,
             vocab_valid: int, dbias: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Single-shard CE forward and backward in one pass (TP 1: the shard is the whole vocab, so
    the row's lse is local): returns the :func:`ce_fwd_stats` rows and overwrites ``logits``
    with :func:`ce_bwd`'s (softmax - onehot) * gscale[row] (+ the column sums into ``dbias``)."""
    stats = ce_fwd_stats(logits, targets, vocab_start, vocab_valid)
    lse = stats[:, 0] + torch.log(stats[:, 1])
    ce_bwd(logits, targets, lse, gscale, vocab_start, vocab_valid, logits, dbias)
    return stats


# -------------------------------------------------------------------------- Adam ----

def adam_step(params, grads, exp_avgs, exp_avg_sqs, shadows, lr: float, beta1: float,
              beta2: float, eps: float, weight_decay: float, step: int, grad_scale: float = 1.0):
    """In-place Adam (torch.optim.Adam semantics, L2 ``weight_decay`` added to the gradient
    as in ``torch.optim.Adam``); also refreshes optional low-precision shadow copies."""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    for i, p in enumerate(params):
        g = grads[i].float() * grad_scale
        if weight_decay != 0:
            g = g + weight_decay * p
        m, v = exp_avgs[i], exp_avg_sqs[i]
        m.mul_(beta1).add_(g, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)
        if shadows is not None and shadows[i] is not None:
            shadows[i].copy_(p)
