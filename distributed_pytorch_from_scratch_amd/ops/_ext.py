"""Loader for the in-tree native extension ``distributed_pytorch_from_scratch_amd._C``.

The extension holds every hand-written HIP/CDNA4 kernel (``csrc/kernels/*.hip``, built for
gfx950 by ``python tools/build_ext.py`` / ``__graft_entry__.build()``).  There is exactly
one compute path per device:

* ``cuda`` (HIP) tensors -> ``_C`` kernels.  If the extension is missing or fails to load,
  ops raise immediately (``require()``): there is no silent eager fallback on the GPU.
* CPU tensors -> ``ops/reference.py`` (pure PyTorch fp32).  That path exists for the
  CPU/gloo plumbing config and as the numerical oracle of every kernel test.
"""
from __future__ import annotations

import importlib
import os

_C = None
_ERR: Exception | None = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    name = "_C_kassert" if kernel_assert() else "_C"
    try:
        _C = importlib.import_module("distributed_pytorch_from_scratch_amd." + name)
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e
        return
    # The attention kernel generation is a per-call argument (``impl`` of attn_fwd / attn_bwd,
    # 0 = the per-head-dim default, the measured winner).  For same-box A/B runs of whole models
    # DPFS_ATTN_IMPL = "<fwd>[,<bwd>]", read once here, becomes the default of that argument.
    if os.environ.get("DPFS_GEMM_GROUP_M"):   # A/B: tile-row group of the GEMMs' item order (4)
        _C.gemm4_group_m(int(os.environ["DPFS_GEMM_GROUP_M"]))
    spec = (os.environ.get("DPFS_ATTN_IMPL") or "0").split(",")
    fi, bi = int(spec[0] or 0), int(spec[1] if len(spec) > 1 and spec[1] else 0)
    if fi or bi:
        _C = _AttnImplDefaults(_C, fi, bi)


def available() -> bool:
    _load()
    return _C is not None


_PROXY = None


def require():
    """Return the native module or raise a loud error (used by every GPU op).

    With ``DPFS_SYNC_DEBUG=1`` or ``DPFS_NAN_CHECK=1`` the module comes wrapped in
    :class:`_DebugProxy`."""
    global _PROXY
    _load()
    if _C is None:
        raise RuntimeError(
            "distributed_pytorch_from_scratch_amd._C (HIP kernels for gfx950) is not built or "
            f"failed to load: {_ERR!r}. Run `python tools/build_ext.py"
            f"{' --kernel-assert' if kernel_assert() else ''}` "
            "(or __graft_entry__.build()).")
    if debug_sync() or nan_check():
        if _PROXY is None:
            _PROXY = _DebugProxy(_C)
        return _PROXY
    return _C


def check_device_errors() -> None:
    """Raise if a kernel reported an error through a host-mapped word (read without a device
    sync): the stream-K GEMM's bounded producer wait timed out, so that GEMM's output is wrong
    (``gemm4.hip`` ``sk_wait``).  The word is sticky; it is reset once reported."""
    if _C is None or not hasattr(_C, "gemm_sk_error"):
        return
    if _C.gemm_sk_error(True):
        raise RuntimeError("stream-K GEMM: a consumer workgroup's wait for its producer's fp32 partial timed out "
                           "(2 s); the GEMM output of that launch is invalid")


def so_path() -> str | None:
    _load()
    return getattr(_C, "__file__", None) if _C is not None else None


def kernel_assert() -> bool:
    """``DPFS_KERNEL_ASSERT=1``: load the bounds-assert build ``_C_kassert`` (built by
    ``python tools/build_ext.py --kernel-assert``) instead of ``_C``; there is no fallback to the
    unchecked build."""
    return os.environ.get("DPFS_KERNEL_ASSERT", "0") == "1"


def debug_sync() -> bool:
    return os.environ.get("DPFS_SYNC_DEBUG", "0") == "1"


def nan_check() -> bool:
    return os.environ.get("DPFS_NAN_CHECK", "0") == "1"


class _AttnImplDefaults:
    """The native module with fixed default ``impl`` arguments for attn_fwd / attn_bwd (an
    explicit ``impl=`` still wins); everything else passes through."""

    def __init__(self, mod, fwd_impl: int, bwd_impl: int):
        self._mod, self._fi, self._bi = mod, fwd_impl, bwd_impl

    def attn_fwd(self, *args, **kw):
        kw.setdefault("impl", self._fi)
        return self._mod.attn_fwd(*args, **kw)

    def attn_bwd(self, *args, **kw):
        kw.setdefault("impl", self._bi)
        return self._mod.attn_bwd(*args, **kw)

    def __getattr__(self, name):
        return getattr(self._mod, name)


class _DebugProxy:
    """Kernel-level debug mode (SURVEY.md §5 "race detection / sanitizers").

    * ``DPFS_SYNC_DEBUG=1``: every op synchronises the device after its launch. A fault or
      launch error is reported against the op that caused it, with its argument shapes,
      instead of surfacing at some later synchronisation. This is the launch-blocking mode.
    * ``DPFS_NAN_CHECK=1``: the floating-point tensor outputs of every op are checked, and
      so are its in-place-written arguments. The first op that produces a NaN/Inf raises.

    Both modes are slow and meant for debugging only.
    """

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn):
            return fn
        import torch

        def desc(args):
            return ", ".join(f"{tuple(a.shape)}:{str(a.dtype).replace('torch.', '')}"
                             if isinstance(a, torch.Tensor) else type(a).__name__ for a in args)

        def wrapped(*args, **kw):
            out = fn(*args, **kw)
            if debug_sync():
                try:
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    raise RuntimeError(f"HIP kernel op `{name}`({desc(args)}) failed: {e}") from e
            if nan_check():
                outs = list(out) if isinstance(out, (list, tuple)) else [out]
                cands = outs + [a for a in args if isinstance(a, torch.Tensor)]
                for t in cands:
                    if isinstance(t, torch.Tensor) and t.is_floating_point() and t.numel() and \
                            not bool(torch.isfinite(t).all()):
                        raise FloatingPointError(f"op `{name}`({desc(args)}) produced non-finite values")
            return out
        return wrapped
