"""Loader for the in-tree native extension ``distributed_pytorch_from_scratch_amd._C``.

The extension holds every hand-written HIP/CDNA4 kernel (``csrc/kernels/*.hip``, built for
gfx950 by ``setup.py build_ext --inplace`` / ``__graft_entry__.build()``).  There is exactly
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
    try:
        _C = importlib.import_module("distributed_pytorch_from_scratch_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e


def available() -> bool:
    _load()
    return _C is not None


def require():
    """Return the native module or raise a loud error (used by every GPU op)."""
    _load()
    if _C is None:
        raise RuntimeError(
            "distributed_pytorch_from_scratch_amd._C (HIP kernels for gfx950) is not built or "
            f"failed to load: {_ERR!r}. Run `python setup.py build_ext --inplace` "
            "(or __graft_entry__.build()).")
    return _C


def so_path() -> str | None:
    _load()
    return getattr(_C, "__file__", None) if _C is not None else None


def debug_sync() -> bool:
    return os.environ.get("DPFS_SYNC_DEBUG", "0") == "1"
