"""MI355X-native tensor-parallel transformer training framework.

Capabilities of ``ldh127/distributed_pytorch_from_scratch`` (Megatron-style TP layers, autograd
collectives, LLaMA-style decoder, train/eval entrypoints, per-rank checkpoints), rebuilt for
AMD Instinct MI355X (gfx950): hand-written HIP/CDNA4 kernels in ``csrc/`` (MFMA GEMMs, flash
attention, fused norms/RoPE/SwiGLU/embedding/vocab-parallel CE/Adam), RCCL over xGMI through
``torch.distributed`` with one process per GPU.
"""
__version__ = "0.1.0"
