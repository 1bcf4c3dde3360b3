from . import reference
from . import functional
from .dispatch import K, shadow
from . import _ext
