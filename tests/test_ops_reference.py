"""The pure-PyTorch oracle kernels (CPU path) against torch autograd.

These are the numerical references of every HIP kernel test, so their backward formulas are
checked here against autograd of the straightforward forward.
"""
import math

import torch
import torch.nn.functional as F

from distributed_pytorch_from_scratch_amd.ops import reference as R


def test_rmsnorm_bwd_matches_autograd():
    torch.manual_seed(0)
    x = torch.randn(7, 32, dtype=torch.float64, requires_grad=True)
    w = torch.rand(32, dtype=torch.float64, requires_grad=True)
    y = w * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5))
    dy = torch.randn_like(y)
    y.backward(dy)
    _, rstd = R.rmsnorm_fwd(x.detach(), w.detach(), 1e-5)
    dx, dw = R.rmsnorm_bwd(dy, x.detach(), w.detach(), rstd)
    assert torch.allclose(dx.double(), x.grad, atol=1e-5) and torch.allclose(dw.double(), w.grad, atol=1e-5)


def test_layernorm_matches_torch():
    torch.manual_seed(1)
    x = torch.randn(5, 24, requires_grad=True)
    w, b = torch.rand(24, requires_grad=True), torch.randn(24, requires_grad=True)
    y = F.layer_norm(x, (24,), w, b, 1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr, mu, rs = R.layernorm_fwd(x.detach(), w.detach(), b.detach(), 1e-5)
    assert torch.allclose(yr, y.detach(), atol=1e-5)
    dx, dw, db = R.layernorm_bwd(dy, x.detach(), w.detach(), mu, rs)
    assert torch.allclose(dx, x.grad, atol=1e-5) and torch.allclose(dw, w.grad, atol=1e-4)
    assert torch.allclose(db, b.grad, atol=1e-5)


def test_swiglu_bwd():
    torch.manual_seed(2)
    gu = torch.randn(6, 16, dtype=torch.float64, requires_grad=True)
    h = F.silu(gu[:, :8]) * gu[:, 8:]
    dh = torch.randn_like(h)
    h.backward(dh)
    assert torch.allclose(R.swiglu_bwd(dh, gu.detach()), gu.grad, atol=1e-10)


def test_rope_matches_reference_formula_and_inverse():
    torch.manual_seed(3)
    M, H, hd = 10, 2, 16
    qkv = torch.randn(M, 3 * H * hd, dtype=torch.float64)
    pos = torch.randint(0, 50, (M,))
    tab = R.rope_table(64, hd, 10000.0).double()
    out = R.rope_(qkv.clone(), pos, tab, 2 * H, hd)
    # reference formula (models/model.py:17-31) with duplicated cos/sin halves
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2).float() / hd))
    ang = pos.float()[:, None] * inv
    cos, sin = torch.cos(ang).repeat(1, 2).double(), torch.sin(ang).repeat(1, 2).double()
    x = qkv[:, : 2 * H * hd].view(M, 2 * H, hd)
    rot = torch.cat([-x[..., hd // 2:], x[..., : hd // 2]], -1)
    ref = x * cos[:, None] + rot * sin[:, None]
    assert torch.allclose(out[:, : 2 * H * hd].view(M, 2 * H, hd), ref, atol=1e-6)
    back = R.rope_(out.clone(), pos, tab, 2 * H, hd, inverse=True)
    assert torch.allclose(back, qkv, atol=1e-6)


def test_attention_matches_sdpa_and_grads():
    torch.manual_seed(4)
    B, T, H, hd = 2, 9, 3, 8
    q, k, v = (torch.randn(B, T, H, hd, dtype=torch.float64, requires_grad=True) for _ in range(3))
    scale = 1 / math.sqrt(hd)
    ref = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                         is_causal=True).transpose(1, 2)
    o, lse = R.attn_fwd(q.detach(), k.detach(), v.detach(), scale, True)
    assert torch.allclose(o.double(), ref.detach(), atol=1e-6)
    do = torch.randn_like(ref)
    ref.backward(do)
    dq, dk, dv = (torch.empty(B, T, H, hd, dtype=torch.float64) for _ in range(3))
    R.attn_bwd(do, q.detach(), k.detach(), v.detach(), o, lse, scale, True, dq, dk, dv)
    assert torch.allclose(dq, q.grad, atol=1e-6) and torch.allclose(dk, k.grad, atol=1e-6)
    assert torch.allclose(dv, v.grad, atol=1e-6)


def test_embedding_oracle():
    w = torch.randn(10, 4)
    ids = torch.tensor([0, 5, 12, 19, 3])
    out = R.embedding_fwd(ids, w, 10, torch.float32)   # shard holds ids [10, 20)
    assert torch.equal(out[2], w[2]) and torch.equal(out[3], w[9]) and out[0].abs().sum() == 0
    dw = R.embedding_bwd(torch.ones(5, 4), ids, 10, 10)
    assert dw[2].sum() == 4 and dw[9].sum() == 4 and dw.sum() == 8


def test_vocab_parallel_ce_oracle_matches_full_ce():
    torch.manual_seed(5)
    M, V, n = 13, 40, 4
    logits = torch.randn(M, V)
    tgt = torch.randint(0, V, (M,))
    shards = logits.chunk(n, dim=1)
    stats = torch.stack([R.ce_fwd_stats(s, tgt, i * (V // n), V // n) for i, s in enumerate(shards)])
    lse, tl = R.ce_combine(stats)
    assert torch.allclose(lse - tl, F.cross_entropy(logits, tgt, reduction="none"), atol=1e-5)


def test_adam_oracle_matches_torch():
    torch.manual_seed(6)
    p = torch.randn(20)
    ref = p.clone().requires_grad_(True)
    m, v = torch.zeros(20), torch.zeros(20)
    opt = torch.optim.Adam([ref], lr=1e-2, betas=(0.9, 0.99), weight_decay=0.1)
    for step in range(1, 5):
        g = torch.randn(20)
        ref.grad = g.clone()
        opt.step()
        R.adam_step([p], [g], [m], [v], None, 1e-2, 0.9, 0.99, 1e-8, 0.1, step)
    assert torch.allclose(p, ref.detach(), atol=1e-6)
