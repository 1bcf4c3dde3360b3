"""Per-shape choice between our MFMA GEMM kernels and hipBLASLt for *plain* GEMMs.

Our kernels (``csrc/kernels/gemm.hip``) carry every GEMM with a fused epilogue: RoPE in the QKV
projection, the fp32 split-K weight-gradient GEMMs that accumulate in place. For the remaining
plain bf16 GEMMs (the forward projections with at most a bias, and the NN data-gradient GEMMs),
the first call on a new (layout, M, N, K, bias) shape times both implementations on the live
operands. Every later call uses the faster one. hipBLASLt is reached through ``torch.nn.functional.linear`` /
``torch.matmul``, with a bias epilogue where there is a bias. The measured per-shape winners are
in ``choices()`` and in ``profiles/``.

``DPFS_GEMM_BACKEND`` = ``auto`` (default) | ``ours`` | ``blas`` pins the choice (tests pin
``ours`` to exercise the HIP kernels).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Tuple

import torch
import torch.nn.functional as F

from . import fp8 as F8
from . import reference
from .dispatch import shadow

_choice: Dict[Tuple, str] = {}
_times: Dict[Tuple, Tuple[float, float]] = {}   # key -> (ours ms, hipBLASLt ms) at selection


def mode() -> str:
    return os.environ.get("DPFS_GEMM_BACKEND", "auto")


def choices(with_times: bool = False) -> Dict[Tuple, object]:
    if with_times:
        return {k: (c,) + tuple(round(t, 4) for t in _times.get(k, ())) for k, c in _choice.items()}
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


def _pick(key: Tuple, ours: Callable, blas: Callable) -> str:
    c = _choice.get(key)
    if c is None:
        # two interleaved rounds, best of each: robust to a collective running alongside
        t_o = min(_ms(ours), _ms(ours))
        t_b = min(_ms(blas), _ms(blas))
        c = "blas" if t_b < 0.97 * t_o else "ours"
        _choice[key] = c
        _times[key] = (t_o, t_b)
    return c


# Below this many rows (decode steps, tiny batches) our 256-row tiles are mostly padding and
# the library's GEMV-class kernels win; timing cannot tell them apart there (a launch-bound
# loop measures the host launch cost, which favours the thinner pybind path).
_MIN_ROWS = 256


def _aligned(*dims: int) -> bool:
    """Our MFMA kernels stage 16-byte rows: every K / N (and TN's M) must be a multiple of 8.
    Uneven vocab shards (e.g. 1000 over 2 ranks at vocab_pad_to=1) go to hipBLASLt."""
    return all(d % 8 == 0 for d in dims)


def gemm_nt(k, x: torch.Tensor, w: torch.Tensor, bias=None, out=None) -> torch.Tensor:
    """y[M,N] = x[M,K] w[N,K]^T (+ bias fp32[N]) in x.dtype (into ``out`` when given: e.g. a
    staging slot of the xGMI collectives, so the collective needs no copy-in)."""
    fw = F8.lookup(w)
    if fw is not None:          # fp8 step (ModelArgs.fp8): e4m3 operands, hipBLASLt fp8 GEMM
        return F8.nt(x, fw, bias, out=out)
    m = mode()
    if k is reference or not x.is_cuda or (m == "ours" and _aligned(x.shape[1], w.shape[0])):
        return k.gemm_nt(x, w, bias, out=out)
    bb = shadow(bias, x.dtype) if bias is not None else None

    def blas():
        if out is None:
            return F.linear(x, w, bb)
        if bb is None:
            return torch.mm(x, w.t(), out=out)
        return torch.addmm(bb, x, w.t(), out=out)
    if not _aligned(x.shape[1], w.shape[0]) or x.shape[0] < _MIN_ROWS:
        return blas()

    def ours():
        return k.gemm_nt(x, w, bias, out=out)
    if m == "blas":
        return blas()
    key = ("nt", x.shape[0], w.shape[0], x.shape[1], bias is not None, x.device.index)
    return blas() if _pick(key, ours, blas) == "blas" else ours()


def small_nt(k, x: torch.Tensor, w: torch.Tensor, bias=None, swiglu: bool = False) -> torch.Tensor:
    """Decode-step projection, M <= 16 rows: y = a w^T (+ bias), a = x or, with ``swiglu``,
    silu(gate) * up of the packed x = [gate | up].  The MFMA GEMV-class kernel (gemv16_k,
    csrc/kernels/decode.hip; SwiGLU fused into its operand load) wherever it applies, else
    hipBLASLt after a separate SwiGLU pass.  Not timed per shape: at these sizes a host-timed
    loop measures launch cost (see _MIN_ROWS); the kernel times are in profiles/."""
    if k is reference or not x.is_cuda:
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
    if k is reference or not a.is_cuda or (m == "ours" and _aligned(a.shape[1], b.shape[1])):
        return k.gemm_nn(a, b, out=out)

    def blas():
        return torch.matmul(a, b) if out is None else torch.matmul(a, b, out=out)
    if not _aligned(a.shape[1], b.shape[1]) or a.shape[0] < _MIN_ROWS:
        return blas()

    def ours():
        return k.gemm_nn(a, b, out=out)
    if m == "blas":
        return blas()
    key = ("nn", a.shape[0], b.shape[1], a.shape[1], a.device.index)
    return blas() if _pick(key, ours, blas) == "blas" else ours()


def gemm_nt_rope(k, x: torch.Tensor, w: torch.Tensor, bias, pos, tab, rot_heads: int, hd: int) -> torch.Tensor:
    """Packed QKV projection with rotate-half RoPE on the first ``rot_heads`` heads: our NT
    kernel with the rotation in its epilogue, or hipBLASLt followed by the in-place RoPE
    kernel (timed per shape like every plain GEMM)."""
    fw = F8.lookup(w)
    if fw is not None:          # fp8 step: fp8 GEMM, then the RoPE pass
        y = F8.nt(x, fw, bias)
        k.rope_(y, pos, tab, rot_heads, hd, False)
        return y
    m = mode()
    if k is reference or not x.is_cuda or m == "ours" or not _aligned(x.shape[1], w.shape[0]) \
            or x.shape[0] < _MIN_ROWS:
        return k.gemm_nt(x, w, bias, pos, tab, rot_heads, hd)
    bb = shadow(bias, x.dtype) if bias is not None else None

    def blas():
        y = F.linear(x, w, bb)
        k.rope_(y, pos, tab, rot_heads, hd)
        return y

    def ours():
        return k.gemm_nt(x, w, bias, pos, tab, rot_heads, hd)
    if m == "blas":
        return blas()
    key = ("nt_rope", x.shape[0], w.shape[0], x.shape[1], hd, x.device.index)
    return blas() if _pick(key, ours, blas) == "blas" else ours()


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
    """fp32 c[M,N] (+)= a[K,M]^T b[K,N] (weight gradients): our split-K kernel or hipBLASLt
    with fp32 output, timed per (shape, accumulate) on a scratch output (an accumulating
    candidate must not be timed into the live gradient)."""
    if k is reference or not a.is_cuda:
        return k.gemm_tn(a, b, out, accumulate) if out is not None else k.gemm_tn(a, b)
    if not _aligned(a.shape[1], b.shape[1]):
        c = torch.matmul(a.t(), b).float()
        if out is None:
            return c
        if accumulate:
            return out.add_(c)
        return out.copy_(c)

    def run(kind, dst, acc):
        if kind == "blas":
            return _blas_tn(a, b, dst, acc)
        return k.gemm_tn(a, b, dst, acc) if dst is not None else k.gemm_tn(a, b)
    m = mode()
    if m == "ours" or a.shape[0] < _MIN_ROWS or not _tn_blas_ok(a, b):
        return run("ours", out, accumulate)
    if m == "blas":
        return run("blas", out, accumulate)
    key = ("tn", a.shape[1], b.shape[1], a.shape[0], bool(accumulate), a.device.index)
    c = _choice.get(key)
    if c is None:
        scratch = torch.zeros(a.shape[1], b.shape[1], device=a.device, dtype=torch.float32)
        c = _pick(key, lambda: run("ours", scratch, accumulate), lambda: run("blas", scratch, accumulate))
    return run(c, out, accumulate)
