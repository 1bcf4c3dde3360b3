"""Reference-compatible import path: ``import ...process_manager as pm; pm.pgm``.

Reference parity: ``process_manager.py`` (module global ``pgm``, ``init_pgm``).  The
implementation is ``parallel/process_manager.py``; attribute access is forwarded so that
``pm.pgm`` always reflects the current manager.
"""
import sys as _sys
from .parallel import process_manager as _impl

_sys.modules[__name__] = _impl
