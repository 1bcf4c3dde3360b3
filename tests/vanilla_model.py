"""Single-device, plain-PyTorch oracle of the reference architecture.

The reference's end-to-end test imports a ``VallinaTransformer`` that does not exist
(``tests/test_transformers.py:14``).  This is that missing oracle, written
from the reference's documented semantics (``models/model.py``): nn.Linear/nn.Embedding,
rotate-half RoPE with duplicated cos/sin halves, materialised causal softmax with a
``-1e4`` masked fill, SwiGLU, pre-norm residuals, untied lm_head.  Initialisation consumes
the RNG in the reference order so that, under the same seed, it equals a TP=k model.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class VRMSNorm(nn.Module):
    def __init__(self, d, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.scale = nn.Parameter(torch.ones(d))

    def forward(self, x):
        xf = x.float()
        return self.scale * (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)).type_as(x)


def _rot(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


class VAttention(nn.Module):
    def __init__(self, d, H):
        super().__init__()
        self.H, self.hd = H, d // H
        self.wq, self.wk, self.wv, self.wo = (nn.Linear(d, d) for _ in range(4))

    def forward(self, x, cos, sin):
        b, t, _ = x.shape
        q, k, v = (l(x).view(b, t, self.H, self.hd).transpose(1, 2) for l in (self.wq, self.wk, self.wv))
        c, s = cos[:, None], sin[:, None]
        q, k = q * c + _rot(q) * s, k * c + _rot(k) * s
        a = (q @ k.transpose(-1, -2)) / math.sqrt(self.hd)
        mask = torch.triu(torch.ones(t, t, dtype=torch.bool, device=x.device), 1)
        a = a.masked_fill(mask, -10000.0).softmax(-1)
        o = (a @ v).transpose(1, 2).reshape(b, t, -1)
        return self.wo(o)


class VFFN(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.gate_proj, self.up_proj, self.down_proj = nn.Linear(d, f), nn.Linear(d, f), nn.Linear(f, d)

    def forward(self, x):
        return self.down_proj(F.silu(self.gate_proj(x)) * self.up_proj(x))


class VLayer(nn.Module):
    def __init__(self, d, f, H):
        super().__init__()
        self.attn, self.ffn = VAttention(d, H), VFFN(d, f)
        self.norm1, self.norm2 = VRMSNorm(d), VRMSNorm(d)

    def forward(self, x, cos, sin):
        x = x + self.attn(self.norm1(x), cos, sin)
        return x + self.ffn(self.norm2(x))


class VanillaTransformer(nn.Module):
    def __init__(self, attn_dim, ffn_dim, num_heads, num_layers, vocab_size, maxlen=2048, rope_theta=1e4):
        super().__init__()
        self.embedding = nn.Embedding(vocab_size, attn_dim)
        self.layers = nn.ModuleList(VLayer(attn_dim, ffn_dim, num_heads) for _ in range(num_layers))
        self.norm = VRMSNorm(attn_dim)
        self.lm_head = nn.Linear(attn_dim, vocab_size)
        hd = attn_dim // num_heads
        theta = 1.0 / (rope_theta ** (torch.arange(0, hd, 2, dtype=torch.int64).float() / hd))
        pos = torch.arange(maxlen).float().unsqueeze(1)
        self.cos = torch.cos(pos * theta).repeat(1, 2)
        self.sin = torch.sin(pos * theta).repeat(1, 2)

    @torch.no_grad()
    def reset_parameters(self):
        def lin(l):
            nn.init.kaiming_uniform_(l.weight, a=math.sqrt(5))
            nn.init.zeros_(l.bias)
        nn.init.normal_(self.embedding.weight, 0.0, 1.0)
        for L in self.layers:
            for l in (L.attn.wq, L.attn.wk, L.attn.wv, L.attn.wo, L.ffn.gate_proj, L.ffn.up_proj, L.ffn.down_proj):
                lin(l)
        lin(self.lm_head)

    def forward(self, ids, pos):
        x = self.embedding(ids)
        cos, sin = self.cos[pos], self.sin[pos]
        for L in self.layers:
            x = L(x, cos, sin)
        return self.lm_head(self.norm(x))
