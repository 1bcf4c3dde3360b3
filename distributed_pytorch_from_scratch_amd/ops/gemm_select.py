"""Per-shape choice among our MFMA GEMM kernels (``csrc/kernels/gemm4.hip``, ``gemm.hip``).

Every GEMM of the training step runs on our kernels: the forward projections (bias, RoPE in
the QKV epilogue), the NN data-gradient GEMMs and the fp32 split-K weight-gradient GEMMs
(reference ``models/layers.py:49,93`` and their autograd backward).  The first call on a new
(layout, M, N, K, bias) shape times our variants on the live operands and every later call
uses the fastest:

* ``ours``     -- the v4 kernel (one wave per SIMD, 128-row wave tiles) with its per-shape
  tile width (256 x 256, or 256 x 192 where whole rounds of tiles over the CUs come out
  shorter, e.g. the N = 768 projections);
* ``ours256`` / ``ours192`` -- v4 with the tile width forced (kept only if it measures faster
  than the width the launcher's round model picked);
* ``ours_nt`` / ``ours256_nt`` / ``ours192_nt`` -- the same with the bf16 output written by
  non-temporal stores (the output streams past L2 instead of displacing the operands the next
  tiles re-read; plain NT / NN outputs);
* ``ours3``    -- the v3 kernel (8 waves, 128 x 64 per wave).

hipBLASLt stays reachable for A/B runs and for operands our kernels do not take (a
contiguous dimension that is not a multiple of 8, e.g. an uneven vocab shard): ``DPFS_GEMM_LIB=1``
adds it to the ``auto`` candidates (``blas``: through ``torch.nn.functional.linear`` /
``torch.matmul`` / ``torch.mm(out_dtype=fp32)``; ``ltN``: algorithm N of its heuristic list
through ``csrc/blas/blaslt.hip``), where it must beat ours by 3 % to be chosen.

``DPFS_GEMM_BACKEND`` = ``auto`` (default) | ``ours`` | ``blas`` | ``lt`` pins the choice.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from . import fp8 as F8
from . import reference
from .dispatch import shadow

_choice: Dict[Tuple, str] = {}
_times: Dict[Tuple, Dict[str, float]] = {}   # key -> {candidate: ms} at selection

# A/B hook for tools/ab_attr.py (same-box interleaved bench runs), not a user switch: False
# turns the grouped weight-gradient launch (gemm_tn_group) off.
TN_GROUP = True


def _direct(k) -> bool:
    """A kernel set whose ops are called as they are, without per-shape candidate timing: the
    CPU oracle (``reference``) and the fp32 kernel set (``fp32_native``, one kernel per op)."""
    return k is reference or getattr(k, "DIRECT", False)


def mode() -> str:
    return os.environ.get("DPFS_GEMM_BACKEND", "auto")


def choices(with_times: bool = False) -> Dict[Tuple, object]:
    if with_times:
        return {k: (c, {n: round(t, 4) for n, t in _times.get(k, {}).items()}) for k, c in _choice.items()}
    return dict(_choice)


def _ms(fn: Callable[[], torch.Tensor], reps: int = 3) -> float:
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


_LT_FINALISTS = 2


def _lib() -> bool:
    """hipBLASLt among the ``auto`` candidates (opt-in A/B: DPFS_GEMM_LIB=1)."""
    return os.environ.get("DPFS_GEMM_LIB", "0") == "1"


def _lt_count(k, layout: int, M: int, N: int, K: int, bias: bool) -> int:
    """Algorithms hipBLASLt offers for this problem through our binding (0: none / disabled)."""
    if not _lib() or not hasattr(k, "lt_algos"):
        return 0
    return int(k.lt_algos(layout, M, N, K, bias))


def _pick(key: Tuple, cands: Dict[str, Callable], lt_count: Callable[[], int] = lambda: 0,
          lt_mk: Optional[Callable[[int], Callable]] = None) -> str:
    c = _choice.get(key)
    if c is None:
        cands = dict(cands)
        n = lt_count() if lt_mk is not None else 0
        if n > 0:
            quick = []
            for i in range(n):
                try:
                    quick.append((_ms(lt_mk(i), reps=2), i))
                except RuntimeError:      # an algorithm the library rejects at run time
                    continue
            for _, i in sorted(quick)[:_LT_FINALISTS]:
                cands[f"lt{i}"] = lt_mk(i)
        # two rounds per candidate, best of each: robust to a collective running alongside
        times = {name: min(_ms(fn), _ms(fn)) for name, fn in cands.items()}
        c = min(times, key=times.get)
        ours_t = {n: t for n, t in times.items() if n.startswith("ours")}
        if not c.startswith("ours") and ours_t:
            best = min(ours_t, key=ours_t.get)
            if times[c] >= 0.97 * ours_t[best]:
                c = best
        _choice[key] = c
        _times[key] = times
    return c


def _lt_index(c: str) -> int:
    return int(c[2:])


# Per-call kernel variant of our GEMM entry points (an argument, never process state):
# 0 = v4 at its per-shape tile width, 1 / 2 = v4 with the 256 / 192 width forced, 3 = v3.
_VARIANT = {"ours": 0, "ours256": 1, "ours192": 2, "ours3": 3, "ours_nt": 4, "ours256_nt": 5, "ours192_nt": 6,
            "ours_sk": 8, "ours_sk_nt": 12}


def _ours_variants(call: Callable[[int], torch.Tensor], widths: bool = False, sk: bool = False) -> Dict[str, Callable]:
    """Our candidates for one call: ``ours`` = the v4 kernel (one wave per SIMD, 128-row wave
    tiles, csrc/kernels/gemm4.hip) at its per-shape tile width and, with ``widths`` (non-split
    bf16 NT / NN), ``ours256`` / ``ours192`` = v4 with the width forced; with ``sk`` (the shape
    has 256-wide tiles at exactly 1.5 per CU) the stream-K kernel ``ours_sk`` as well.  The v3
    kernel (variant 3) lost to v4 on every step shape (profiles/r3_gemm_v4_probe_salu.txt) and
    is no longer a candidate; it remains the fallback for shapes the v4 launcher declines."""
    out = {"ours": lambda: call(0)}
    if widths:
        out.update({"ours256": lambda: call(1), "ours192": lambda: call(2)})
        if NT_STORES:
            out.update({"ours_nt": lambda: call(4), "ours256_nt": lambda: call(5), "ours192_nt": lambda: call(6)})
    if widths and sk:
        out.update({"ours_sk": lambda: call(8)})
        if NT_STORES:
            out["ours_sk_nt"] = lambda: call(12)
    return out


# A/B hook (tools/ab_attr.py): the non-temporal-store variants among the per-shape candidates.
# They are timed alone, where an output that streams past the caches can only help; in the
# step the next kernel then reads that output from HBM instead of the infinity cache.
NT_STORES = True


def _sk_ok(k, M: int, N: int, K: int) -> bool:
    """Whether the stream-K bf16 kernel is a candidate for this NT / NN shape on this device:
    it applies (256 x 256 tiles at 1.5 per CU) and K is long enough for its one fp32 partial
    hand-off to undercut the split-K slabs (SK_MIN_K)."""
    return STREAM_K and K >= SK_MIN_K and hasattr(k, "gemm_sk_applies") and bool(k.gemm_sk_applies(M, N, K))


# A/B hook (tools/ab_attr.py): the stream-K kernel among the per-shape candidates.  At K <= 4096
# it ties or loses to the 192-wide kernel (the hand-off's latency, profiles/r5_stream_k.txt),
# so only the long-K shapes (the lm_head data gradient, K = vocab) try it, against split-K.
STREAM_K = True
SK_MIN_K = 8192


def _run_ours(call: Callable[[int], torch.Tensor], choice: str):
    return call(_VARIANT.get(choice, 0))


# Below this many rows (decode steps, tiny batches) a host-timed loop measures launch cost, not
# the kernels: no per-shape timing there, the default variant runs.
_MIN_ROWS = 256


def _aligned(*dims: int) -> bool:
    """Our bf16 MFMA kernels stage 16-byte rows: every K / N (and TN's M) must be a multiple of
    8.  Other shapes (e.g. an uneven vocab shard, 1000 over 2 ranks at vocab_pad_to=1) run
    :func:`_unaligned`."""
    return all(d % 8 == 0 for d in dims)


def _rm(t: torch.Tensor) -> torch.Tensor:
    return t if t.dim() == 2 and t.stride(1) == 1 else t.contiguous()


def _unaligned(k, layout: int, a: torch.Tensor, b: torch.Tensor, bias=None, out=None, accumulate: bool = False):
    """A GEMM whose K / N is not a multiple of 8: the fp32-input MFMA kernel (``gemm_f32``,
    csrc/kernels/fp32.hip) reading the bf16 operands at any alignment (converted to fp32 as
    they are staged; exact products, fp32 accumulate, fp32 bias in the epilogue, split-K for
    the long-K weight gradients).  ``DPFS_GEMM_LIB=blas`` pins torch's library GEMM instead."""
    if mode() == "blas":
        return None
    o = out if out is None or out.stride(-1) == 1 else None
    c = k.gemm_f32(_rm(a), _rm(b), layout, bias, o, bool(accumulate and o is not None))
    if out is not None and o is None:
        return out.add_(c) if accumulate else out.copy_(c)
    return c


def _lt_operands_ok(*ts) -> bool:
    return all(t is None or (t.is_contiguous() and t.dtype == torch.bfloat16) for t in ts)


def _lt_bias_ok(bias) -> bool:
    return bias is None or (bias.dtype == torch.float32 and bias.is_contiguous())


def gemm_nt(k, x: torch.Tensor, w: torch.Tensor, bias=None, out=None) -> torch.Tensor:
    """y[M,N] = x[M,K] w[N,K]^T (+ bias fp32[N]) in x.dtype (into ``out`` when given: e.g. a
    staging slot of the xGMI collectives, so the collective needs no copy-in)."""
    fw = F8.lookup(w)
    if fw is not None:          # fp8 step (ModelArgs.fp8): e4m3 operands, hipBLASLt fp8 GEMM
        return F8.nt(x, fw, bias, out=out)
    m = mode()
    if _direct(k) or not x.is_cuda or (m in ("ours", "auto") and _aligned(x.shape[1], w.shape[0])
                                           and x.shape[0] < _MIN_ROWS) or \
            (m == "ours" and _aligned(x.shape[1], w.shape[0])):
        return k.gemm_nt(x, w, bias, out=out)
    bb = shadow(bias, x.dtype) if bias is not None else None

    def blas():
        if out is None:
            return F.linear(x, w, bb)
        if bb is None:
            return torch.mm(x, w.t(), out=out)
        return torch.addmm(bb, x, w.t(), out=out)
    if not _aligned(x.shape[1], w.shape[0]):
        y = _unaligned(k, 0, x, w, bias, out)
        return blas() if y is None else y
    M, N, K = x.shape[0], w.shape[0], x.shape[1]
    lt_ok = _lt_operands_ok(x, w, out) and _lt_bias_ok(bias)

    def lt(i):
        def run():
            y = out if out is not None else torch.empty(M, N, device=x.device, dtype=x.dtype)
            k.lt_run(0, x, w, y, bias, i)
            return y
        return run

    def ours(variant: int = 0):
        return k.gemm_nt(x, w, bias, out=out, variant=variant)
    if m == "blas":
        return blas()
    if m == "lt":
        return lt(0)() if lt_ok and _lt_count(k, 0, M, N, K, bias is not None) else blas()
    key = ("nt", M, N, K, bias is not None, x.device.index)
    c = _pick(key, {**_ours_variants(ours, True, _sk_ok(k, M, N, K)), **({"blas": blas} if _lib() else {})},
              lambda: _lt_count(k, 0, M, N, K, bias is not None), lt if lt_ok else None)
    if c.startswith("ours") or (c != "blas" and not lt_ok):   # (an lt choice needs contiguous operands)
        return _run_ours(ours, c)
    return blas() if c == "blas" else lt(_lt_index(c))()


def swiglu_epilogue(k, w: torch.Tensor, want: Optional[bool] = None) -> bool:
    """Whether the gate|up projection of packed weight ``w`` [2F, d] runs with SwiGLU in its GEMM
    epilogue (``gate_up``).  ``want`` = ``ModelArgs.swiglu_epilogue``: None (default) = on the
    GPU kernels (not with a pinned library backend or the fp8 step), off on the CPU oracle;
    True runs the interleaved layout on the CPU oracle too (tests of its plumbing); False
    turns it off."""
    if w.size(0) % 128 or want is False:
        return False
    if _direct(k) or not w.is_cuda:
        return bool(want)
    return mode() in ("auto", "ours") and F8.lookup(w) is None and hasattr(k, "gemm_nt_swiglu")


def gate_up(k, x: torch.Tensor, w: torch.Tensor, b, perm: bool):
    """(gu, h = silu(gate) * up) of the gate|up projection (w / b natural [gate | up]).
    ``perm``: the GEMM reads the weight rows interleaved in 64-row blocks (reference.gu_perm)
    and writes h from its epilogue (gemm_nt_swiglu); gu comes out interleaved and the backward
    reads it with ``swiglu_bwd(..., perm=True)``, which returns the natural-layout gradient.
    Where the fused kernel declines the shape, an interleaved copy of the weight, the plain
    GEMM and the interleaved SwiGLU pass give the same tensors."""
    if perm:
        r = k.gemm_nt_swiglu(x, w, b)
        if r:
            return r[0], r[1]
        gu = gemm_nt(k, x, reference.gu_perm(w).contiguous(),
                     reference.gu_perm(b).contiguous() if b is not None else None)
        return gu, k.swiglu_fwd(gu, True)
    gu = gemm_nt(k, x, w, b)
    return gu, k.swiglu_fwd(gu)


def down_dgrad_swiglu(k, dy: torch.Tensor, w: torch.Tensor, gu: torch.Tensor, dbias, perm: bool) -> torch.Tensor:
    """d gate|up (natural layout) = SwiGLU'(gu) * (dy w): the down projection's data gradient
    with the SwiGLU backward in the GEMM epilogue (gemm_nn_swiglu_bwd: dy w never reaches
    memory; the gate|up bias gradient comes from the same kernel into ``dbias``).  Falls back to
    gemm_nn + swiglu_bwd where the fused kernel declines the shape, for the fp8 step or a pinned
    library backend (profiles/r4_swiglu_bwd_epilogue_ab.txt: the fused form is 0.40 ms/step
    faster)."""
    fused = (not _direct(k) and dy.is_cuda and mode() in ("auto", "ours") and F8.lookup(w, dgrad=True) is None
             and hasattr(k, "gemm_nn_swiglu_bwd"))
    if fused:
        r = k.gemm_nn_swiglu_bwd(dy, w, gu, dbias, perm)
        if r:
            return r[0]
    return k.swiglu_bwd(gemm_nn(k, dy, w), gu, dbias, perm)


def small_nt(k, x: torch.Tensor, w: torch.Tensor, bias=None, swiglu: bool = False) -> torch.Tensor:
    """Decode-step projection, M <= 16 rows: y = a w^T (+ bias), a = x or, with ``swiglu``,
    silu(gate) * up of the packed x = [gate | up].  The MFMA GEMV-class kernel (gemv16_k,
    csrc/kernels/decode.hip; SwiGLU fused into its operand load) wherever it applies, else
    hipBLASLt after a separate SwiGLU pass.  Not timed per shape: at these sizes a host-timed
    loop measures launch cost (see _MIN_ROWS); the kernel times are in profiles/."""
    if _direct(k) or not x.is_cuda:
        return k.gemv_nt(x, w, bias, swiglu)
    if mode() != "blas" and k.gemv_nt_ok(x, w, swiglu):
        return k.gemv_nt(x, w, bias, swiglu)
    return gemm_nt(k, k.swiglu_fwd(x) if swiglu else x, w, bias)


def gemm_nn(k, a: torch.Tensor, b: torch.Tensor, out=None) -> torch.Tensor:
    """c[M,N] = a[M,K] b[K,N] in a.dtype (into ``out`` when given)."""
    fw = F8.lookup(b, dgrad=True)
    if fw is not None:          # fp8 step: e5m2 gradient x e4m3 weight
        return F8.nn(a, fw, out=out)
    m = mode()
    if _direct(k) or not a.is_cuda or (m in ("ours", "auto") and _aligned(a.shape[1], b.shape[1])
                                           and a.shape[0] < _MIN_ROWS) or \
            (m == "ours" and _aligned(a.shape[1], b.shape[1])):
        return k.gemm_nn(a, b, out=out)

    def blas():
        return torch.matmul(a, b) if out is None else torch.matmul(a, b, out=out)
    if not _aligned(a.shape[1], b.shape[1]):
        y = _unaligned(k, 1, a, b, None, out)
        return blas() if y is None else y
    M, N, K = a.shape[0], b.shape[1], a.shape[1]
    lt_ok = _lt_operands_ok(a, b, out)

    def lt(i):
        def run():
            y = out if out is not None else torch.empty(M, N, device=a.device, dtype=a.dtype)
            k.lt_run(1, a, b, y, None, i)
            return y
        return run

    def ours(variant: int = 0):
        return k.gemm_nn(a, b, out=out, variant=variant)
    if m == "blas":
        return blas()
    if m == "lt":
        return lt(0)() if lt_ok and _lt_count(k, 1, M, N, K, False) else blas()
    key = ("nn", M, N, K, a.device.index)
    c = _pick(key, {**_ours_variants(ours, True, _sk_ok(k, M, N, K)), **({"blas": blas} if _lib() else {})},
              lambda: _lt_count(k, 1, M, N, K, False), lt if lt_ok else None)
    if c.startswith("ours") or (c != "blas" and not lt_ok):   # (an lt choice needs contiguous operands)
        return _run_ours(ours, c)
    return blas() if c == "blas" else lt(_lt_index(c))()


def gemm_nt_rope(k, x: torch.Tensor, w: torch.Tensor, bias, pos, tab, rot_heads: int, hd: int) -> torch.Tensor:
    """Packed QKV projection with rotate-half RoPE on the first ``rot_heads`` heads: our NT
    kernel with the rotation in its epilogue (v4 or v3, timed per shape); with
    ``DPFS_GEMM_LIB=1`` also hipBLASLt followed by the in-place RoPE kernel."""
    fw = F8.lookup(w)
    if fw is not None:          # fp8 step: fp8 GEMM, then the RoPE pass
        y = F8.nt(x, fw, bias)
        k.rope_(y, pos, tab, rot_heads, hd, False)
        return y
    m = mode()
    if not _direct(k) and x.is_cuda and not _aligned(x.shape[1], w.shape[0]):
        y = _unaligned(k, 0, x, w, bias)
        if y is None:
            y = F.linear(x, w, shadow(bias, x.dtype) if bias is not None else None)
        k.rope_(y, pos, tab, rot_heads, hd, False)
        return y
    if _direct(k) or not x.is_cuda or m == "ours" or x.shape[0] < _MIN_ROWS:
        return k.gemm_nt(x, w, bias, pos, tab, rot_heads, hd)
    bb = shadow(bias, x.dtype) if bias is not None else None
    M, N, K = x.shape[0], w.shape[0], x.shape[1]
    lt_ok = _lt_operands_ok(x, w) and _lt_bias_ok(bias)

    def blas():
        y = F.linear(x, w, bb)
        k.rope_(y, pos, tab, rot_heads, hd)
        return y

    def lt(i):
        def run():
            y = torch.empty(M, N, device=x.device, dtype=x.dtype)
            k.lt_run(0, x, w, y, bias, i)
            k.rope_(y, pos, tab, rot_heads, hd)
            return y
        return run

    def ours(variant: int = 0):
        return k.gemm_nt(x, w, bias, pos, tab, rot_heads, hd, variant=variant)

    # The rotated Q|K columns and the V columns as two launches into one output: at GPT-2
    # small's 2304 columns one launch is 1152 tiles of 256 x 256 = 4.5 rounds of the CUs, the
    # pair 768 tiles (3 rounds) + 512 tiles of 256 x 192 (2 rounds of 3/4 the work).
    rot = rot_heads * hd
    # (only where the rotation is fused into the Q|K launch's epilogue: the separate RoPE pass
    # of other head dims needs a contiguous output)
    split_ok = hd in (64, 128) and 0 < rot < N and rot % 256 == 0 and (N - rot) % 64 == 0 and \
        w.is_contiguous() and (bias is None or bias.is_contiguous())

    def ours_split():
        y = torch.empty(M, N, device=x.device, dtype=x.dtype)
        k.gemm_nt(x, w[:rot], bias[:rot] if bias is not None else None, pos, tab, rot_heads, hd, out=y[:, :rot])
        k.gemm_nt(x, w[rot:], bias[rot:] if bias is not None else None, out=y[:, rot:])
        return y
    if m == "blas":
        return blas()
    if m == "lt":
        return lt(0)() if lt_ok and _lt_count(k, 0, M, N, K, bias is not None) else blas()
    # (rot and split_ok in the key: a cached ``ours_split`` choice is only reused where the
    # split form applies to this call)
    key = ("nt_rope", M, N, K, hd, rot, split_ok, x.device.index)
    c = _pick(key, {**_ours_variants(ours), **({"ours_split": ours_split} if split_ok else {}),
                    **({"blas": blas} if _lib() else {})},
              lambda: _lt_count(k, 0, M, N, K, bias is not None), lt if lt_ok else None)
    if c == "ours_split" and split_ok:
        return ours_split()
    if c.startswith("ours") or (c != "blas" and not lt_ok):   # (an lt choice needs contiguous operands)
        return _run_ours(ours, c)
    return blas() if c == "blas" else lt(_lt_index(c))()


_TN_BLAS = {}   # device index -> whether hipBLASLt's bf16 x bf16 -> fp32 mm works on this build


def _blas_tn(a: torch.Tensor, b: torch.Tensor, out, accumulate: bool) -> torch.Tensor:
    """hipBLASLt fp32-output wgrad: c[M,N] (+)= a[K,M]^T b[K,N] via aten mm/addmm(out_dtype)."""
    at = a.t()
    if out is None:
        return torch.mm(at, b, out_dtype=torch.float32)
    if accumulate:
        return torch.addmm(out, at, b, out_dtype=torch.float32, out=out)
    return torch.mm(at, b, out_dtype=torch.float32, out=out)


def _tn_blas_ok(a, b) -> bool:
    dev = a.device.index
    ok = _TN_BLAS.get(dev)
    if ok is None:
        try:   # functional probe on a small problem against an fp32 matmul (incl. accumulate)
            g = torch.Generator(device=a.device).manual_seed(0)
            pa = torch.randn(96, 32, device=a.device, generator=g).to(a.dtype)
            pb = torch.randn(96, 40, device=a.device, generator=g).to(a.dtype)
            ref = pa.float().t() @ pb.float()
            c = _blas_tn(pa, pb, None, False)
            c2 = _blas_tn(pa, pb, c.clone(), True)
            ok = c.dtype == torch.float32 and bool(torch.allclose(c, ref, atol=1e-2, rtol=1e-3)) and \
                bool(torch.allclose(c2, 2 * ref, atol=2e-2, rtol=1e-3))
        except Exception:   # this torch / ROCm build has no bf16 -> fp32 mm: ours only
            ok = False
        _TN_BLAS[dev] = ok
    return ok


def gemm_tn(k, a: torch.Tensor, b: torch.Tensor, out=None, accumulate: bool = False) -> torch.Tensor:
    """fp32 c[M,N] (+)= a[K,M]^T b[K,N] (weight gradients): our split-K kernel (v4 / v3), and
    with ``DPFS_GEMM_LIB=1`` hipBLASLt through torch (fp32 output) or directly (accumulating
    in place, beta = 1), timed per (shape, accumulate) on a scratch output (an accumulating
    candidate must not be timed into the live gradient)."""
    if _direct(k) or not a.is_cuda:
        return k.gemm_tn(a, b, out, accumulate) if out is not None else k.gemm_tn(a, b)
    if not _aligned(a.shape[1], b.shape[1]):
        c = _unaligned(k, 2, a, b, None, out, accumulate)
        if c is not None:
            return c
        c = torch.matmul(a.t(), b).float()
        if out is None:
            return c
        if accumulate:
            return out.add_(c)
        return out.copy_(c)
    M, N, K = a.shape[1], b.shape[1], a.shape[0]
    lt_ok = _lt_operands_ok(a, b) and (out is None or out.is_contiguous())

    def run(kind, dst, acc):
        if kind == "blas":
            return _blas_tn(a, b, dst, acc)
        if kind.startswith("lt"):
            if dst is None:
                dst, acc = torch.empty(M, N, device=a.device, dtype=torch.float32), False
            k.lt_run(2, a, b, dst, None, _lt_index(kind), acc)
            return dst
        v = _VARIANT.get(kind, 0)
        return k.gemm_tn(a, b, dst, acc, variant=v) if dst is not None else k.gemm_tn(a, b, variant=v)
    m = mode()
    if m == "ours" or a.shape[0] < _MIN_ROWS:
        return run("ours", out, accumulate)
    blas_ok = (m == "blas" or _lib()) and _tn_blas_ok(a, b)
    if m == "blas" and blas_ok:
        return run("blas", out, accumulate)
    if m == "lt":
        ok = lt_ok and _lt_count(k, 2, M, N, K, False) > 0
        return run("lt0" if ok else "ours", out, accumulate)
    key = ("tn", M, N, K, bool(accumulate), a.device.index)
    c = _choice.get(key)
    if c is None:
        scratch = torch.zeros(M, N, device=a.device, dtype=torch.float32)
        cands = {"ours": lambda: run("ours", scratch, accumulate)}
        if blas_ok and _lib():
            cands["blas"] = lambda: run("blas", scratch, accumulate)
        c = _pick(key, cands, lambda: _lt_count(k, 2, M, N, K, False),
                  (lambda i: (lambda: run(f"lt{i}", scratch, accumulate))) if lt_ok else None)
    if c.startswith("lt") and not lt_ok:
        c = "ours"
    return run(c, out, accumulate)


def gemm_tn_pair(k, a0: torch.Tensor, b0: torch.Tensor, a1: torch.Tensor, b1: torch.Tensor, out=None,
                 accumulate: bool = False) -> torch.Tensor:
    """fp32 c (+)= a0^T b0 + a1^T b1 -- a weight gradient over the two ping-pong chunks of a
    chunked step.  Candidates, timed per shape like the others: ``pair`` = ONE split-K launch
    whose K-splits read either chunk's buffers and ONE slab reduction (``gemm_tn2``: the plan
    of a single tall GEMM), ``split`` = two :func:`gemm_tn` calls (two under-filled grids,
    two reductions)."""
    def split(dst, acc):
        c = gemm_tn(k, a0, b0, dst, acc)
        return gemm_tn(k, a1, b1, c, True)

    if _direct(k) or not a0.is_cuda or not hasattr(k, "gemm_tn2") or mode() not in ("auto", "ours"):
        return split(out, accumulate)
    M, N = a0.shape[1], b0.shape[1]
    if not _aligned(M, N) or min(a0.shape[0], a1.shape[0]) < _MIN_ROWS:
        return split(out, accumulate)
    key = ("tn2", M, N, a0.shape[0], a1.shape[0], bool(accumulate), a0.device.index)
    c = _choice.get(key)
    if c is None:
        scratch = torch.zeros(M, N, device=a0.device, dtype=torch.float32)
        if k.gemm_tn2(a0, b0, a1, b1, scratch, accumulate) is None:    # the K-split plan does not fit
            c = _choice[key] = "split"
        else:
            c = _pick(key, {"split": lambda: split(scratch, accumulate),
                            "pair": lambda: k.gemm_tn2(a0, b0, a1, b1, scratch, accumulate)})
    if c == "pair":
        r = k.gemm_tn2(a0, b0, a1, b1, out, accumulate)
        if r is not None:
            return r
    return split(out, accumulate)


def gemm_tn_group(k, items) -> list:
    """Several weight gradients over the same rows, ``items`` = [(a, b, out, accumulate)] or
    [(a, b, out, accumulate, a1, b1)] (a chunked step: the rows continue in the other ping-pong
    chunk's buffers): out (+)= a^T b (+ a1^T b1) each.  Candidates, timed per group shape:
    ``group`` = ONE persistent 32x32x16 launch over every GEMM's tiles with one shared K-split
    length and one slab reduction (``gemm_tn_group``: the launches' ramps / tails and per-GEMM
    slab round trips of the separate calls are paid once; with two buffers the split length
    divides the first one's rows, so no work item straddles them), ``each`` = one
    :func:`gemm_tn` (:func:`gemm_tn_pair`) per item."""
    items = [tuple(it) + (None, None) if len(it) == 4 else tuple(it) for it in items]
    two = items[0][4] is not None
    outs = [it[2] for it in items]

    def each(dsts):
        if two:
            return [gemm_tn_pair(k, a, b, a1, b1, d, acc) for (a, b, _, acc, a1, b1), d in zip(items, dsts)]
        return [gemm_tn(k, a, b, d, acc) for (a, b, _, acc, _, _), d in zip(items, dsts)]

    if (not TN_GROUP or _direct(k) or len(items) < 2 or any(o is None for o in outs) or not items[0][0].is_cuda
            or not hasattr(k, "gemm_tn_group") or mode() not in ("auto", "ours")
            or any((it[4] is not None) != two for it in items)):
        return each(outs)
    K = items[0][0].shape[0]
    K1 = items[0][4].shape[0] if two else 0
    if K < _MIN_ROWS or any(it[0].shape[0] != K or it[1].shape[0] != K for it in items) or \
            (two and any(it[4].shape[0] != K1 or it[5].shape[0] != K1 for it in items)):
        return each(outs)
    A = [it[0] for it in items]
    B = [it[1] for it in items]
    A2 = [it[4] for it in items] if two else None
    B2 = [it[5] for it in items] if two else None
    acc = [int(bool(it[3])) for it in items]
    key = ("tng",) + tuple((a.shape[1], b.shape[1], bool(x)) for a, b, _, x, _, _ in items) + (K, K1, A[0].device.index)
    c = _choice.get(key)
    if c is None:
        scratch = [torch.zeros(a.shape[1], b.shape[1], device=a.device, dtype=torch.float32) for a, b in zip(A, B)]
        if not k.gemm_tn_group(A, B, scratch, acc, A2, B2):     # the group does not apply to these shapes
            c = _choice[key] = "each"
        else:
            c = _pick(key, {"each": lambda: each(scratch), "group": lambda: k.gemm_tn_group(A, B, scratch, acc, A2, B2)})
    if c == "group" and k.gemm_tn_group(A, B, outs, acc, A2, B2):
        return outs
    return each(outs)
