"""Special tokens, ignore index and the default model configuration.

Reference parity: ``constants.py:1-17`` (``BOS_TOKEN``/``EOS_TOKEN``/``UNK_TOKEN``,
``IGNORE_INDEX = -1``, ``ModelArgumments``).  The model config lives in
``models/config.py`` (``ModelArgs``; ``ModelArgumments`` is kept as an alias).
"""
from .models.config import ModelArgs, ModelArgumments  # noqa: F401

BOS_TOKEN = "<BOS>"
EOS_TOKEN = "<EOS>"
UNK_TOKEN = "<UNK>"
IGNORE_INDEX = -1
