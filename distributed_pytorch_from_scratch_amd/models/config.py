"""Model configurations and presets.

``ModelArgs`` defaults are the reference's ``ModelArgumments`` (``constants.py:9-17``):
d=512, ffn=2048, 8 heads, RoPE theta 1e4, 12 layers, vocab 1024, maxlen 1000 — a
51,473,920-parameter LLaMA-style decoder with biased linears and an untied lm_head.

Presets (``BASELINE.json`` configs) keep the reference block (pre-norm, RoPE, SwiGLU, untied
head) and pick the published model shapes:

=============  =====  ====  =====  =====  ======  ======  ====================================
preset         d      L     heads  ffn    vocab   maxlen  note
=============  =====  ====  =====  =====  ======  ======  ====================================
reference      512    12    8      2048   1024    1000    reference default (51.47M params)
plumbing       128    2     4      512    1024    256     BASELINE config 1 (CPU/gloo)
gpt2-small     768    12    12     2048   50257   1024    SwiGLU 3x768x2048 = GPT-2 MLP 2x768x3072
gpt2-large     1280   36    20     3456   50257   1024    SwiGLU ffn ~= 2/3 * 5120, 128-aligned
llama2-7b      4096   32    32     11008  32000   4096    no biases (LLaMA-2 shape)
llama-13b      5120   40    40     13824  32000   8192    BASELINE config 5 (seq 8192)
=============  =====  ====  =====  =====  ======  ======  ====================================

The vocabulary is padded to a multiple of ``vocab_pad_to`` (128 -> 50304 for GPT-2, which
also divides by 1/2/4/8) for MFMA-friendly lm_head shards; padded columns are masked out
of the softmax and sliced off any returned logits.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, replace
from typing import Dict, Optional


@dataclass
class ModelArgs:
    attn_dim: int = 512
    ffn_dim: int = 2048
    num_heads: int = 8
    rope_theta: float = 10000.0
    num_layers: int = 12
    vocab_size: int = 1024
    maxlen: int = 1000
    # --- extensions (defaults reproduce the reference) ---
    bias: bool = True
    norm: str = "rmsnorm"            # "rmsnorm" | "layernorm"
    norm_eps: float = 1e-5
    vocab_pad_to: int = 128
    sequence_parallel: bool = False
    # When the heads do not divide over the TP ranks (12 heads at TP 8: 2 on ranks 0-3, 1 on
    # ranks 4-7), give the lighter ranks a larger vocabulary shard so every rank carries the
    # same work (vocab_partition).  Off, or with an even head split, the reference's vocab
    # ranges are used (equal shards, remainder on the last rank: layers.py:120-132).
    vocab_balance: bool = True
    # Activation recompute in the explicit-schedule engines: keep only each layer's input and
    # re-run the layer forward (collectives included) in backward.  ~16x less activation
    # memory per layer at GPT-2 width for ~1/3 more compute (long-sequence / large configs).
    recompute: bool = False
    # fp8 GEMMs in the explicit-schedule engines (ops/fp8.py): forward and data-gradient
    # projections with per-tensor e4m3 / e5m2 operands on hipBLASLt's fp8 kernels; weight
    # gradients, attention, norms and the optimizer stay bf16 / fp32.  Off by default.
    fp8: bool = False
    # SwiGLU in the gate|up GEMM epilogue (weight rows read interleaved in 64-row blocks,
    # ops/gemm_select.swiglu_epilogue): None = on for the GPU kernels, off on the CPU oracle;
    # True also runs the interleaved layout on the CPU oracle (tests of its plumbing).
    swiglu_epilogue: Optional[bool] = None

    @property
    def head_dim(self) -> int:
        return self.attn_dim // self.num_heads

    @property
    def padded_vocab_size(self) -> int:
        m = max(1, self.vocab_pad_to)
        return ((self.vocab_size + m - 1) // m) * m

    def num_params(self) -> int:
        d, f, L, V = self.attn_dim, self.ffn_dim, self.num_layers, self.padded_vocab_size
        b = 1 if self.bias else 0
        per_layer = 4 * d * d + 3 * d * f + b * (3 * d + d + 2 * f + d) + 2 * d * (2 if self.norm == "layernorm" else 1)
        return V * d * 2 + b * V + L * per_layer + d * (2 if self.norm == "layernorm" else 1)

    def matmul_params(self) -> int:
        """Parameters that take part in a GEMM per token (6N FLOP basis): every linear incl.
        the lm_head, excluding the embedding lookup."""
        d, f, L, V = self.attn_dim, self.ffn_dim, self.num_layers, self.padded_vocab_size
        return L * (4 * d * d + 3 * d * f) + V * d

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token: 6 * matmul params + causal attention (fwd+bwd)."""
        attn = 12 * self.num_layers * self.attn_dim * seq_len / 2  # causal -> half of T^2
        return 6 * self.matmul_params() + attn


def vocab_partition(args: "ModelArgs", head_sizes, granule: int = 64):
    """Per-rank vocab shard sizes for a TP group whose ranks hold ``head_sizes`` heads.

    Each rank's step work ~ heads_r * W_head + vocab_r * W_col with, per token and layer,
    W_head = 24 d hd (QKV + Wo GEMMs, fwd + bwd) + 21 T hd (causal attention fwd + bwd, counted
    at 1/3 of GEMM efficiency) and W_col = 6 d / L (lm_head GEMMs).  Ranks with fewer heads get
    (h_max - h_r) * W_head / W_col extra columns; shards are multiples of ``granule`` (the
    last rank takes the remainder).  Even head splits keep the reference ranges."""
    n = len(head_sizes)
    V = args.padded_vocab_size
    per = V // n
    ref = [per] * (n - 1) + [V - per * (n - 1)]
    if n == 1 or not args.vocab_balance or len(set(head_sizes)) == 1 or V < 4 * granule * n:
        return ref
    d, hd, L = args.attn_dim, args.head_dim, args.num_layers
    T = min(args.maxlen, 2048)
    cols_per_head = L * (24 * d * hd + 21 * T * hd) / (6 * d)
    hmax = max(head_sizes)
    extra = [(hmax - h) * cols_per_head for h in head_sizes]
    base = (V - sum(extra)) / n
    if base < granule:                       # vocab too small to balance fully: scale down
        f = (V - granule * n) / max(1.0, sum(extra))
        extra = [e * f for e in extra]
        base = (V - sum(extra)) / n
    sizes = [max(granule, int(round((base + e) / granule)) * granule) for e in extra[:-1]]
    last = V - sum(sizes)
    if last < granule // 2:
        return ref
    return sizes + [last]


# Backwards-compatible alias with the reference's (misspelt) name.
ModelArgumments = ModelArgs

PRESETS: Dict[str, ModelArgs] = {
    "reference": ModelArgs(),
    "plumbing": ModelArgs(attn_dim=128, ffn_dim=512, num_heads=4, num_layers=2, vocab_size=1024,
                          maxlen=256),
    "gpt2-small": ModelArgs(attn_dim=768, ffn_dim=2048, num_heads=12, num_layers=12,
                            vocab_size=50257, maxlen=1024),
    "gpt2-large": ModelArgs(attn_dim=1280, ffn_dim=3456, num_heads=20, num_layers=36,
                            vocab_size=50257, maxlen=1024),
    "llama2-7b": ModelArgs(attn_dim=4096, ffn_dim=11008, num_heads=32, num_layers=32,
                           vocab_size=32000, maxlen=4096, bias=False),
    "llama-13b": ModelArgs(attn_dim=5120, ffn_dim=13824, num_heads=40, num_layers=40,
                           vocab_size=32000, maxlen=8192, bias=False),
}


def get_preset(name: str, **overrides) -> ModelArgs:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; choose from {sorted(PRESETS)}")
    return replace(PRESETS[name], **overrides)


def to_dict(a: ModelArgs) -> dict:
    return asdict(a)
