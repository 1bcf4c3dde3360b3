"""HIP kernel numerics vs the plain-PyTorch fp32 oracle (``ops/reference.py``), on MI355X.

Every test runs the ``_C`` kernel on ``cuda`` tensors and the reference on the same inputs
upcast to fp32; tolerances are bf16-rounding sized.  Shapes include ragged edges (M, N not
multiples of the 128x128 GEMM tile, T not a multiple of the attention tiles).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed_pytorch_from_scratch_amd.ops import _ext, reference as R  # noqa: E402


@pytest.fixture(scope="module")
def C():
    return _ext.require()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


DEV = "cuda"


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (1000, 768, 768), (33, 200, 64), (4096, 2304, 768),
                                   (130, 6288, 768), (512, 96, 1024)])
def test_gemm_nt(C, M, N, K):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    out = C.gemm_nt(a, b, bias)
    ref = R.gemm_nt(a.float(), b.float(), bias)
    assert _rel(out, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (1000, 768, 2304), (33, 64, 200), (4096, 768, 288)])
def test_gemm_nn(C, M, N, K):
    torch.manual_seed(1)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16()
    out = C.gemm_nn(a, b)
    assert _rel(out, R.gemm_nn(a.float(), b.float())) < 1e-2


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (2304, 768, 4096), (96, 768, 1000), (200, 64, 33)])
def test_gemm_tn(C, M, N, K):
    torch.manual_seed(2)
    a = torch.randn(K, M, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16()
    out = C.gemm_tn(a, b)
    assert out.dtype == torch.float32
    assert _rel(out, R.gemm_tn(a.float(), b.float())) < 1e-2
    acc = torch.randn(M, N, device=DEV)
    acc_ref = acc.clone() + R.gemm_tn(a.float(), b.float())
    C.gemm_tn(a, b, acc, True)
    assert _rel(acc, acc_ref) < 1e-2


def test_gemm_identity_asymmetric(C):
    # A = I with an asymmetric B catches a transposed C write (guide §3).
    n = 128
    eye = torch.eye(n, device=DEV).bfloat16()
    b = torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n).remainder(251).bfloat16()
    out = C.gemm_nt(eye, b, None)          # = b^T
    assert torch.equal(out.float(), b.float().t())
    out = C.gemm_nn(eye, b)                # = b
    assert torch.equal(out.float(), b.float())


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,D", [(37, 768), (1024, 512), (5, 5120), (64, 128)])
def test_rmsnorm(C, dt, M, D):
    torch.manual_seed(3)
    x = torch.randn(M, D, device=DEV).to(dt)
    w = torch.rand(D, device=DEV) + 0.5
    y, rstd = C.rmsnorm_fwd(x, w, 1e-5)
    yr, rr = R.rmsnorm_fwd(x.float(), w, 1e-5)
    assert _rel(y, yr) < 1e-2 and _rel(rstd, rr) < 1e-5
    dy = torch.randn(M, D, device=DEV).to(dt)
    dx, dw = C.rmsnorm_bwd(dy, x, w, rstd)
    dxr, dwr = R.rmsnorm_bwd(dy.float(), x.float(), w, rr)
    assert _rel(dx, dxr) < 1e-2 and _rel(dw, dwr) < 1e-3


@pytest.mark.parametrize("M,D", [(37, 768), (300, 1280)])
def test_layernorm(C, M, D):
    torch.manual_seed(4)
    x = torch.randn(M, D, device=DEV).bfloat16()
    w, b = torch.rand(D, device=DEV) + 0.5, torch.randn(D, device=DEV)
    y, mu, rs = C.layernorm_fwd(x, w, b, 1e-5)
    yr, mur, rsr = R.layernorm_fwd(x.float(), w, b, 1e-5)
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(M, D, device=DEV).bfloat16()
    dx, dw, db = C.layernorm_bwd(dy, x, w, mu, rs)
    dxr, dwr, dbr = R.layernorm_bwd(dy.float(), x.float(), w, mur, rsr)
    assert _rel(dx, dxr) < 1e-2 and _rel(dw, dwr) < 1e-3 and _rel(db, dbr) < 1e-3


def test_rmsnorm_bwd_deterministic(C):
    x = torch.randn(4096, 768, device=DEV).bfloat16()
    w = torch.rand(768, device=DEV)
    y, r = C.rmsnorm_fwd(x, w, 1e-5)
    dy = torch.randn_like(x)
    a = C.rmsnorm_bwd(dy, x, w, r)[1]
    b = C.rmsnorm_bwd(dy, x, w, r)[1]
    assert torch.equal(a, b)


def test_swiglu(C):
    torch.manual_seed(5)
    gu = torch.randn(333, 2 * 1024, device=DEV).bfloat16()
    h = C.swiglu_fwd(gu)
    assert _rel(h, R.swiglu_fwd(gu.float())) < 1e-2
    dh = torch.randn(333, 1024, device=DEV).bfloat16()
    assert _rel(C.swiglu_bwd(dh, gu), R.swiglu_bwd(dh.float(), gu.float())) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("hd", [16, 32, 48, 64, 128])
def test_rope(C, hd, dtype):
    """Vectorised kernel (hd/2 a multiple of the 16-byte vector) and the scalar fallback
    (bf16 hd 48), both against the fp32 reference; the inverse rotation restores the input."""
    torch.manual_seed(6)
    M, H = 1000, 3
    qkv = torch.randn(M, 3 * H * hd, device=DEV).to(dtype)
    pos = torch.randint(0, 200, (M,), device=DEV)
    tab = R.rope_table(256, hd, 10000.0).to(DEV)
    a = qkv.clone()
    C.rope_(a, pos, tab, 2 * H, hd, False)
    b = qkv.float().clone()
    R.rope_(b, pos, tab, 2 * H, hd, False)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert _rel(a, b) < tol
    assert torch.equal(a[:, 2 * H * hd:], qkv[:, 2 * H * hd:])     # v heads untouched
    C.rope_(a, pos, tab, 2 * H, hd, True)  # inverse restores
    assert _rel(a, qkv) < tol


def test_bias_grad_and_residual(C):
    torch.manual_seed(7)
    dy = torch.randn(1000, 768, device=DEV).bfloat16()
    assert _rel(C.bias_grad(dy), R.bias_grad(dy.float())) < 1e-4
    y = torch.randn(1000, 768, device=DEV).bfloat16()
    res = torch.randn(1000, 768, device=DEV).bfloat16()
    bias = torch.randn(768, device=DEV)
    out = C.bias_residual(y, bias, res)
    assert _rel(out, y.float() + bias + res.float()) < 1e-2
    y2 = y.clone()
    C.add_bias_(y2, bias)
    assert _rel(y2, y.float() + bias) < 1e-2


def test_embedding(C):
    torch.manual_seed(8)
    V, D, M = 1000, 768, 513
    w = torch.randn(V, D, device=DEV)
    ids = torch.randint(0, 3 * V, (M,), device=DEV)
    for st in (0, V, 2 * V):
        out = C.embedding_fwd(ids, w, st, torch.bfloat16)
        ref = R.embedding_fwd(ids, w, st, torch.float32)
        assert _rel(out, ref) < 1e-2
        d = torch.randn(M, D, device=DEV).bfloat16()
        assert _rel(C.embedding_bwd(d, ids, V, st), R.embedding_bwd(d.float(), ids, V, st)) < 1e-3


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("V,D,M", [(1000, 768, 4096), (50304, 768, 32768), (300, 20, 777), (64, 6, 100)])
def test_embedding_bwd_sorted_deterministic(C, V, D, M, dt):
    """The sorted embedding gradient (one wave per vocab row over its segment of the stably
    sorted ids, no atomics): every row written (stale output overwritten, untouched ids zero),
    equal to the fp32 oracle, bit-identical run to run and with the ids in another order of the
    same multiset per row; accumulate adds; vocab shards (ids outside dropped); D % 4 != 0 runs
    the atomic fallback."""
    torch.manual_seed(36)
    d = torch.randn(M, D, device=DEV).to(dt)
    ids = torch.randint(0, 3 * V, (M,), device=DEV)
    ids[: M // 8] = 5 + V                         # a hot token (a long segment)
    for st in (0, V):
        out = torch.full((V, D), float("nan"), device=DEV)
        C.embedding_bwd_sorted(d, ids, V, st, out=out)
        ref = R.embedding_bwd(d.float(), ids, V, st)
        assert torch.isfinite(out).all() and _rel(out, ref) < 1e-5
        out2 = torch.empty(V, D, device=DEV)
        C.embedding_bwd_sorted(d, ids, V, st, out=out2)
        assert torch.equal(out, out2) or D % 4   # (the D % 4 != 0 fallback is the atomic form)
        acc = torch.randn(V, D, device=DEV)
        want = acc + ref
        C.embedding_bwd_sorted(d, ids, V, st, out=acc, accumulate=True)
        assert _rel(acc, want) < 1e-5
    if D % 4 == 0:   # fixed summation order: the row order within an id, not the thread schedule
        a = C.embedding_bwd_sorted(d, ids, V, V)
        assert torch.equal(a, C.embedding_bwd_sorted(d.clone(), ids.clone(), V, V))


@pytest.mark.parametrize("V,valid,start", [(6288, 6288, 0), (6288, 6241, 6288 * 7), (1024, 1000, 0),
                                           (500, 500, 500)])
def test_cross_entropy_kernels(C, V, valid, start):
    torch.manual_seed(9)
    M = 257
    x = (3 * torch.randn(M, V, device=DEV)).bfloat16()
    t = torch.randint(start, start + V, (M,), device=DEV)
    st = C.ce_fwd_stats(x, t, start, valid)
    sr = R.ce_fwd_stats(x.float(), t, start, valid)
    assert _rel(st, sr) < 1e-4
    lse, _ = R.ce_combine(sr.unsqueeze(0))
    g = torch.rand(M, device=DEV)
    out = torch.empty_like(x)
    C.ce_bwd(x, t, lse, g, start, valid, out)
    ref = torch.empty(M, V, device=DEV)
    R.ce_bwd(x.float(), t, lse, g, start, valid, ref)
    assert _rel(out, ref) < 1e-2


@pytest.mark.parametrize("B,T,H,hd", [(2, 256, 4, 64), (1, 300, 2, 64), (2, 130, 3, 128), (1, 64, 2, 32),
                                      (1, 1000, 2, 64), (1, 1000, 2, 128), (2, 384, 2, 128)])
@pytest.mark.parametrize("impl", [1, 4, 6, 8, 9])
def test_attention(C, B, T, H, hd, impl):
    # per call: forward 16x16x32 register-staged / 32x32x16 LDS-DMA ring (6: with the row sum by
    # MFMA), backward pair 16x16x32 / 32x32x16 key-on-lane (hd 32 has only the first of each;
    # impl 6 of the backward = the fused head_dim-64 kernel)
    # (impl 8: the forward with the scale and running max folded into its MFMAs)
    # (impl 9 of the backward: the v3 pair with K pre-scaled by scale log2 e)
    if impl in (6, 8, 9) and hd == 32:
        pytest.skip("impl 6 / 8 / 9: head_dim 64 / 128")
    _check_attention(C, B, T, H, hd, 4 if impl == 9 else impl, {1: 2, 4: 4, 6: 6 if hd == 64 else 4, 8: 4, 9: 9}[impl])


def _check_attention(C, B, T, H, hd, fimpl=0, bimpl=0):
    torch.manual_seed(10)
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).bfloat16()
    q = qkv[:, : H * hd].view(B, T, H, hd)
    k = qkv[:, H * hd: 2 * H * hd].view(B, T, H, hd)
    v = qkv[:, 2 * H * hd:].view(B, T, H, hd)
    scale = 1 / math.sqrt(hd)
    o, lse = C.attn_fwd(q, k, v, scale, True, impl=fimpl)
    orf, lser = R.attn_fwd(q.float(), k.float(), v.float(), scale, True)
    assert _rel(o, orf) < 2e-2
    assert (lse - lser).abs().max().item() < 2e-2
    do = torch.randn(B, T, H, hd, device=DEV).bfloat16()
    dqkv = torch.empty_like(qkv)
    dq = dqkv[:, : H * hd].view(B, T, H, hd)
    dk = dqkv[:, H * hd: 2 * H * hd].view(B, T, H, hd)
    dv = dqkv[:, 2 * H * hd:].view(B, T, H, hd)
    C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv, impl=bimpl)
    rq, rk, rv = (torch.empty(B, T, H, hd, device=DEV) for _ in range(3))
    R.attn_bwd(do.float(), q.float(), k.float(), v.float(), o.float(), lse, scale, True, rq, rk, rv)
    assert _rel(dq, rq) < 3e-2 and _rel(dk, rk) < 3e-2 and _rel(dv, rv) < 3e-2


@pytest.mark.parametrize("impl", [1, 4, 6, 8])
@pytest.mark.parametrize("hd", [64, 128])
def test_attention_fwd_rescale_branch(C, impl, hd):
    """The online softmax's deferred rescale fires only when a row's max grows by > 2^8 between
    tiles (data-dependent, rare on random data; guide rule 26): keys whose scores grow along
    the sequence plus isolated spikes force it on many tiles, at rows both inside and at the
    edge of a wave's query block.  Output and LSE against the fp32 oracle."""
    torch.manual_seed(12)
    B, T, H = 2, 640, 3
    q = torch.randn(B, T, H, hd, device=DEV)
    k = torch.randn(B, T, H, hd, device=DEV) * (1 + 6 * torch.arange(T, device=DEV) / T).view(1, T, 1, 1)
    for t in (70, 200, 333, 517, 600):          # spikes aligned with some queries
        k[:, t] = 4 * q[:, t + 3 if t + 3 < T else t]
    v = torch.randn(B, T, H, hd, device=DEV)
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    o, lse = C.attn_fwd(q, k, v, 1 / math.sqrt(hd), True, impl=impl)
    orf, lser = R.attn_fwd(q.float(), k.float(), v.float(), 1 / math.sqrt(hd), True)
    assert _rel(o, orf) < 2e-2, _rel(o, orf)
    assert (lse - lser).abs().max().item() < 5e-2 * max(1.0, lser.abs().max().item() / 10)


def test_attention_deterministic(C):
    B, T, H, hd = 2, 512, 2, 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    o, lse = C.attn_fwd(q, k, v, 0.125, True)
    do = torch.randn_like(o)
    outs = []
    for _ in range(2):
        d = torch.empty_like(qkv)
        dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
        C.attn_bwd(do, q, k, v, o, lse, 0.125, True, dq, dk, dv)
        outs.append(d)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B,T,H", [(2, 1024, 3), (1, 1000, 2), (3, 777, 1), (2, 2048, 2), (1, 192, 2)])
def test_attention_bwd_cross_block_prefetch_is_bit_identical(C, B, T, H):
    """dK/dV at head_dim 64 fetches the second key block's first Q / dO tiles and K / V during
    the first block's last tiles, dQ the second query block's K / V tiles and Q / dO / O rows;
    the arithmetic is unchanged: bit-identical to the cold-prologue forms (each alone and both),
    and against the fp32 oracle (ragged T: partial key blocks and query tiles)."""
    torch.manual_seed(13)
    hd = 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    o, lse = C.attn_fwd(q, k, v, 0.125, True)
    do = torch.randn_like(o)
    outs = []
    try:
        for pf in (3, 0, 1, 2):
            C.attn_prefetch(pf)
            d = torch.empty_like(qkv)
            dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
            C.attn_bwd(do, q, k, v, o, lse, 0.125, True, dq, dk, dv)
            outs.append((d, dq, dk, dv))
    finally:
        C.attn_prefetch(3)
    for x in outs[1:]:
        assert torch.equal(outs[0][0], x[0])
    rq, rk, rv = (torch.empty(B, T, H, hd, device=DEV) for _ in range(3))
    R.attn_bwd(do.float(), q.float(), k.float(), v.float(), o.float(), lse, 0.125, True, rq, rk, rv)
    _, dq, dk, dv = outs[0]
    assert _rel(dq, rq) < 3e-2 and _rel(dk, rk) < 3e-2 and _rel(dv, rv) < 3e-2


@pytest.mark.parametrize("B,T,H,causal", [(2, 1024, 3, True), (1, 1000, 2, True), (3, 777, 1, True),
                                           (1, 192, 2, True), (1, 64, 1, True), (2, 2048, 1, True),
                                           (2, 256, 2, False), (1, 300, 2, False), (1, 130, 1, False)])
def test_attention_bwd_fused6(C, B, T, H, causal):
    """The fused head_dim-64 backward (impl 6: delta pass, one dK / dV / dQ kernel over 256-key
    blocks with dS shared through LDS, deterministic fp32 dQ partial reduction) against the fp32
    oracle, the dQ + dK/dV pair (impl 4) and itself (bitwise, two runs); causal and not,
    ragged T (partial key blocks / query tiles), strided (packed QKV) views."""
    torch.manual_seed(41)
    hd = 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    o, lse = C.attn_fwd(q, k, v, 0.125, causal)
    do = torch.randn_like(o)
    outs = []
    for impl in (6, 6, 4):
        d = torch.full_like(qkv, float("nan"))
        dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
        C.attn_bwd(do, q, k, v, o, lse, 0.125, causal, dq, dk, dv, impl=impl)
        outs.append((d, dq, dk, dv))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.isfinite(outs[0][0].float()).all()
    rq, rk, rv = (torch.empty(B, T, H, hd, device=DEV) for _ in range(3))
    R.attn_bwd(do.float(), q.float(), k.float(), v.float(), o.float(), lse, 0.125, causal, rq, rk, rv)
    _, dq, dk, dv = outs[0]
    assert _rel(dq, rq) < 3e-2 and _rel(dk, rk) < 3e-2 and _rel(dv, rv) < 3e-2, (_rel(dq, rq), _rel(dk, rk), _rel(dv, rv))
    _, dq4, dk4, dv4 = outs[2]
    assert _rel(dq, dq4) < 1e-2 and _rel(dk, dk4) < 1e-2 and _rel(dv, dv4) < 1e-2


@pytest.mark.parametrize("T", [192, 1024, 333])
def test_attention_bwd_fused6_rope_and_bias(C, T):
    """impl 6 with the inverse RoPE (dK in the fused kernel's epilogue, dQ in the partial
    reduction) and the QKV bias gradient (column sums from both) against the oracle."""
    torch.manual_seed(42)
    B, H, hd = 2, 3, 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    o, lse = C.attn_fwd(q, k, v, hd ** -0.5, True)
    do = torch.randn_like(o)
    pos = torch.randint(0, 2048, (B * T,), device=DEV)
    tab = R.rope_table(2048, hd, 10000.0).to(DEV)
    d = torch.empty_like(qkv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    db = torch.full((3 * H * hd,), float("nan"), device=DEV)
    assert C.attn_bwd(do, q, k, v, o, lse, hd ** -0.5, True, dq, dk, dv, pos, tab, dbias=db, impl=6)
    assert _rel(db, d.float().sum(0)) < 5e-3
    r = torch.empty(B * T, 3 * H * hd, device=DEV)
    rq, rk, rv = (r[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    rdb = torch.empty(3 * H * hd, device=DEV)
    R.attn_bwd(do.float(), q.float(), k.float(), v.float(), o.float(), lse, hd ** -0.5, True, rq, rk, rv,
               pos, tab, dbias=rdb)
    assert _rel(d, r) < 3e-2
    assert _rel(db, rdb) < 3e-2


@pytest.mark.parametrize("nsh,M", [(1, 32768), (2, 1000), (8, 4097)])
def test_ce_finalize_and_valid_scale(C, nsh, M):
    """The CE loss bookkeeping kernels (one workgroup, fixed-order sums) against the oracle:
    per-row lse / validity, running sums over two chunks, the mean loss; and the one-pass
    CE's per-row gradient scale."""
    torch.manual_seed(43)
    st = torch.stack([torch.randn(nsh, M, device=DEV) * 3, torch.rand(nsh, M, device=DEV) * 50 + 1,
                      torch.randn(nsh, M, device=DEV)], dim=2).contiguous()
    tgt = torch.randint(0, 100, (M,), device=DEV)
    tgt[::7] = -1
    acc, loss = torch.empty(2, device=DEV), torch.empty((), device=DEV)
    racc, rloss = torch.empty(2, device=DEV), torch.empty((), device=DEV)
    for first, last in ((True, False), (False, True)):
        lse, valid = C.ce_finalize(st, tgt, -1, acc, loss, first, last)
        rl, rv = R.ce_finalize(st, tgt, -1, racc, rloss, first, last)
        assert _rel(lse, rl) < 1e-5 and torch.equal(valid, rv)
    assert _rel(acc, racc) < 1e-5 and abs(loss.item() - rloss.item()) < 1e-4 * abs(rloss.item())
    gs, n = C.ce_valid_scale(tgt, -1)
    rg, rn = R.ce_valid_scale(tgt, -1)
    assert torch.equal(n, rn) and _rel(gs, rg) < 1e-6


@pytest.mark.parametrize("M,V,start", [(32768, 50304, 0), (1000, 1024, 0), (4097, 6288, 6288), (5, 10, 0),
                                       (70000, 12000, 24000)])
def test_emb_sort_matches_stable_sort(C, M, V, start):
    """The embedding backward's radix sort (two 8-bit LSD passes, ballot ranks): the same perm /
    seg as a stable framework sort, with skewed ids (one very frequent row) and ids outside the
    shard; and the sorted backward built on it equals the one built on the framework sort."""
    torch.manual_seed(44)
    ids = torch.randint(0, 3 * V, (M,), device=DEV) if start else torch.randint(0, V, (M,), device=DEV)
    ids[::3] = start + V // 2          # a frequent token
    perm, seg = C.emb_sort(ids, start, V)
    rp, rs = R.emb_sort(ids, start, V)
    assert torch.equal(seg, rs)
    n = int(rs[-1])
    assert torch.equal(perm[:n], rp[:n])
    if M >= 1000:
        d = torch.randn(M, 64, device=DEV).bfloat16()
        a = C.embedding_bwd_sorted(d, ids, V, start, perm=perm, seg=seg)
        b = R.embedding_bwd(d.float(), ids, V, start)
        assert _rel(a, b) < 1e-5


@pytest.mark.parametrize("layout,M,N,K", [(0, 300, 200, 96), (0, 1024, 768, 512), (1, 257, 129, 64), (1, 512, 2048, 768),
                                         (2, 512, 512, 32000), (0, 128, 128, 8192),
                                         (2, 768, 768, 1000), (2, 96, 130, 33), (0, 65, 67, 7)])
def test_gemm_f32(C, layout, M, N, K):
    """fp32-input MFMA GEMM (exact fp32 products, the fp32 training path) in the three layouts
    against float64: bias (NT), accumulate into an existing output (TN), ragged / unaligned
    shapes and a column-slice output."""
    torch.manual_seed(45)
    if layout == 0:
        a, b = torch.randn(M, K, device=DEV), torch.randn(N, K, device=DEV)
        ref = a.double() @ b.double().t()
    elif layout == 1:
        a, b = torch.randn(M, K, device=DEV), torch.randn(K, N, device=DEV)
        ref = a.double() @ b.double()
    else:
        a, b = torch.randn(K, M, device=DEV), torch.randn(K, N, device=DEV)
        ref = a.double().t() @ b.double()
    bias = torch.randn(N, device=DEV) if layout == 0 else None
    c = C.gemm_f32(a, b, layout, bias)
    want = ref + (bias.double() if bias is not None else 0)
    assert (c.double() - want).abs().max().item() < 1e-4 * max(1.0, K ** 0.5)
    if layout == 2:
        acc = torch.randn(M, N, device=DEV)
        want2 = acc.double() + ref
        C.gemm_f32(a, b, 2, None, acc, True)
        assert (acc.double() - want2).abs().max().item() < 1e-4 * max(1.0, K ** 0.5)
    wide = torch.zeros(M, N + 8, device=DEV)
    C.gemm_f32(a, b, layout, bias, wide[:, :N])
    assert torch.equal(wide[:, :N], c) and not wide[:, N:].any()


@pytest.mark.parametrize("layout,M,N,K", [(0, 300, 500, 777), (1, 257, 501, 999), (2, 1003, 501, 4097),
                                          (0, 64, 1000, 768), (2, 768, 1000, 8192)])
def test_gemm_unaligned_bf16(C, layout, M, N, K):
    """bf16 GEMMs whose K / N is not a multiple of 8 (an uneven vocab shard): gemm_select routes
    them to the fp32-input MFMA kernel reading bf16 at any alignment -- no torch matmul.
    Against the fp32 product of the same bf16 values (exact products, fp32 accumulate)."""
    from distributed_pytorch_from_scratch_amd.ops import gemm_select as G
    torch.manual_seed(47)
    bf = torch.bfloat16
    if layout == 0:
        a, b = torch.randn(M, K, device=DEV, dtype=bf), torch.randn(N, K, device=DEV, dtype=bf)
        ref = a.double() @ b.double().t()
        bias = torch.randn(N, device=DEV)
        c = G.gemm_nt(C, a, b, bias)
        ref = ref + bias.double()
    elif layout == 1:
        a, b = torch.randn(M, K, device=DEV, dtype=bf), torch.randn(K, N, device=DEV, dtype=bf)
        ref = a.double() @ b.double()
        c = G.gemm_nn(C, a, b)
    else:
        a, b = torch.randn(K, M, device=DEV, dtype=bf), torch.randn(K, N, device=DEV, dtype=bf)
        ref = a.double().t() @ b.double()
        c = G.gemm_tn(C, a, b)
        assert c.dtype == torch.float32
        acc = torch.randn(M, N, device=DEV)
        want2 = acc.double() + ref
        G.gemm_tn(C, a, b, acc, True)
        assert (acc.double() - want2).abs().max().item() < 1e-4 * K ** 0.5
    tol = (1e-4 if layout == 2 else 1e-2) * K ** 0.5   # bf16 output rounding for NT / NN
    assert (c.double() - ref).abs().max().item() < tol * (1 if layout == 2 else ref.abs().max().item() / K ** 0.5)


@pytest.mark.parametrize("B,T,H,hd,causal", [(2, 256, 2, 64, True), (1, 300, 3, 64, True), (1, 130, 2, 128, True),
                                             (2, 192, 2, 32, True), (1, 200, 2, 64, False)])
def test_attention_f32(C, B, T, H, hd, causal):
    """fp32 flash attention (fp32-input MFMAs) forward / backward against the fp32 oracle,
    packed QKV views, with inverse RoPE and the QKV bias gradient in the backward."""
    torch.manual_seed(46)
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV)
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    scale = hd ** -0.5
    o, lse = C.attn_fwd_f32(q, k, v, scale, causal)
    orf, lser = R.attn_fwd(q, k, v, scale, causal)
    assert _rel(o, orf) < 1e-5 and (lse - lser).abs().max().item() < 1e-4
    do = torch.randn_like(o)
    pos = torch.randint(0, 1024, (B * T,), device=DEV)
    tab = R.rope_table(1024, hd, 10000.0).to(DEV)
    d = torch.empty_like(qkv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    db = torch.full((3 * H * hd,), float("nan"), device=DEV)
    assert C.attn_bwd_f32(do, q, k, v, o, lse, scale, causal, dq, dk, dv, pos, tab, db)
    r = torch.empty(B * T, 3 * H * hd, device=DEV)
    rq, rk, rv = (r[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    rdb = torch.empty(3 * H * hd, device=DEV)
    R.attn_bwd(do, q, k, v, o, lse, scale, causal, rq, rk, rv, pos, tab, dbias=rdb)
    assert _rel(d, r) < 1e-4, _rel(d, r)
    assert _rel(db, rdb) < 1e-4


@pytest.mark.parametrize("layout,M,N,K,variant", [("nn", 32768, 768, 16384, 8), ("nn", 32768, 768, 3072, 0),
                                                  ("nt", 32768, 2304, 768, 0), ("nt", 32768, 768, 2048, 8)])
def test_gemm_beside_collective_standin_is_bitwise(C, layout, M, N, K, variant):
    """The persistent v4 GEMM (static item striding over one workgroup per CU) and the stream-K
    variant (consumers spin on their producer's flag) launched while a collective stand-in
    (tools/tp_sim.py --emulate-comm: 64 resident 1024-thread workgroups, 3 ms) holds CUs on a
    side stream: the output is bit-identical to the undisturbed run and no stream-K wait timed
    out (the displaced workgroups start when the stand-in leaves)."""
    if variant == 8 and not C.gemm_sk_applies(M, N, K):
        pytest.skip("stream-K needs 256 x 256 tiles at exactly 1.5 per CU on this device")
    torch.manual_seed(47)
    a = (torch.randn(M, K, device=DEV) / 8).bfloat16()
    b = (torch.randn(K, N, device=DEV) / 8).bfloat16() if layout == "nn" else (torch.randn(N, K, device=DEV) / 8).bfloat16()
    run = (lambda: C.gemm_nn(a, b, variant=variant)) if layout == "nn" else (lambda: C.gemm_nt(a, b, None, variant=variant))
    C.gemm_sk_error(True)
    ref = run()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    outs = []
    for _ in range(3):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            C.occupy(64, 3000.0)
        outs.append(run())
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)
    assert C.gemm_sk_error(False) == 0


def test_adam_matches_torch(C):
    torch.manual_seed(11)
    ps = [torch.randn(n, device=DEV) for n in (1000, 16384 * 2 + 7, 4096)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    gs = [torch.randn_like(p) for p in ps]
    ms = [torch.zeros_like(p) for p in ps]
    vs = [torch.zeros_like(p) for p in ps]
    sh = [torch.empty_like(p, dtype=torch.bfloat16) for p in ps]
    desc, chunks = C.adam_build(ps, gs, ms, vs, sh)
    opt = torch.optim.Adam(ref, lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)
    for step in range(1, 4):
        for r, g in zip(ref, gs):
            r.grad = g.clone()
        opt.step()
        C.adam_step(desc, chunks, 1e-3, 0.9, 0.95, 1e-8, 0.01, step)
    for p, r, s in zip(ps, ref, sh):
        assert (p - r.detach()).abs().max().item() < 1e-5
        assert torch.equal(s, p.bfloat16())


@pytest.mark.parametrize("M,N,K,heads,hd", [(2048, 2304, 768, 24, 64), (300, 1152, 768, 12, 64),
                                            (4096, 576, 768, 6, 64), (1000, 3072, 1024, 16, 128),
                                            (513, 1536, 512, 8, 128)])
def test_gemm_nt_fused_rope(C, M, N, K, heads, hd):
    """QKV projection with the RoPE rotation in the GEMM epilogue (hd 64 and 128) vs GEMM +
    reference RoPE."""
    torch.manual_seed(12)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=DEV)
    pos = torch.randint(0, 1024, (M,), device=DEV)
    tab = R.rope_table(1024, hd, 10000.0).to(DEV)
    c = C.gemm_nt(a, b, bias, pos, tab, heads, hd)
    ref = a.float() @ b.float().t() + bias
    R.rope_(ref, pos, tab, heads, hd, False)
    assert _rel(c, ref) < 1e-2
    # unrotated tail (v heads) untouched by the rotation
    assert _rel(c[:, heads * hd:], (a.float() @ b.float().t() + bias)[:, heads * hd:]) < 1e-2


@pytest.mark.parametrize("hd", [64, 128])
def test_attention_bwd_fused_inverse_rope(C, hd):
    torch.manual_seed(13)
    B, T, H = 2, 192, 3
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    o, lse = C.attn_fwd(q, k, v, hd ** -0.5, True)
    do = torch.randn_like(o)
    pos = torch.randint(0, 512, (B * T,), device=DEV)
    tab = R.rope_table(512, hd, 10000.0).to(DEV)
    d = torch.empty_like(qkv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    C.attn_bwd(do, q, k, v, o, lse, hd ** -0.5, True, dq, dk, dv, pos, tab)
    r = torch.empty(B * T, 3 * H * hd, device=DEV)
    rq, rk, rv = (r[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    R.attn_bwd(do.float(), q.float(), k.float(), v.float(), o.float(), lse, hd ** -0.5, True, rq, rk, rv)
    R.rope_(r, pos, tab, 2 * H, hd, True)
    assert _rel(d, r) < 3e-2


@pytest.mark.parametrize("hd,T", [(64, 192), (128, 130), (32, 1024)])
def test_attention_bwd_fused_qkv_bias_grad(C, hd, T):
    """dbias = column sums of the stored dq | dk | dv (inverse RoPE applied), from the attention
    backward's epilogues; ragged T masks the rows past the sequence."""
    torch.manual_seed(26)
    B, H = 2, 3
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    o, lse = C.attn_fwd(q, k, v, hd ** -0.5, True)
    do = torch.randn_like(o)
    pos = torch.randint(0, 2048, (B * T,), device=DEV)
    tab = R.rope_table(2048, hd, 10000.0).to(DEV)
    d = torch.empty_like(qkv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    db = torch.full((3 * H * hd,), float("nan"), device=DEV)
    assert C.attn_bwd(do, q, k, v, o, lse, hd ** -0.5, True, dq, dk, dv, pos, tab, dbias=db)
    want = d.float().sum(0)
    assert _rel(db, want) < 5e-3
    r = torch.empty(B * T, 3 * H * hd, device=DEV)
    rq, rk, rv = (r[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    rdb = torch.empty(3 * H * hd, device=DEV)
    R.attn_bwd(do.float(), q.float(), k.float(), v.float(), o.float(), lse, hd ** -0.5, True, rq, rk, rv,
               pos, tab, dbias=rdb)
    assert _rel(db, rdb) < 3e-2


def test_rmsnorm_bwd_fused_residual_grad(C):
    torch.manual_seed(14)
    M, D = 513, 768
    x = torch.randn(M, D, device=DEV).bfloat16()
    w = torch.randn(D, device=DEV)
    dy = torch.randn(M, D, device=DEV).bfloat16()
    dres = torch.randn(M, D, device=DEV).bfloat16()
    _, rstd = C.rmsnorm_fwd(x, w, 1e-5)
    dx, dw = C.rmsnorm_bwd(dy, x, w, rstd, dres)
    rdx, rdw = R.rmsnorm_bwd(dy.float(), x.float(), w, rstd, dres.float())
    assert _rel(dx, rdx) < 1e-2 and _rel(dw, rdw) < 1e-2


@pytest.mark.parametrize("M,F", [(4096, 3072), (333, 1024), (40, 64)])
def test_swiglu_bwd_fused_bias_grad(C, M, F):
    torch.manual_seed(15)
    gu = torch.randn(M, 2 * F, device=DEV).bfloat16()
    dh = torch.randn(M, F, device=DEV).bfloat16()
    db = torch.empty(2 * F, device=DEV)
    dgu = C.swiglu_bwd(dh, gu, db)
    rdb = torch.empty(2 * F, device=DEV)
    rdgu = R.swiglu_bwd(dh.float(), gu.float(), rdb)
    assert _rel(dgu, rdgu) < 1e-2 and _rel(db, rdb) < 1e-3
    assert torch.equal(dgu, C.swiglu_bwd(dh, gu))


@pytest.mark.parametrize("hd", [32, 64, 128])
@pytest.mark.parametrize("L", [0, 255, 256, 699])
def test_decode_attention_and_kv_append(C, hd, L):
    """Split-K single-query attention over a KV cache (csrc/kernels/decode.hip) against the
    fp32 oracle, across split boundaries; kv_append writes row *len; step_advance."""
    torch.manual_seed(21)
    B, H, Tmax = 3, 5, 700
    kc = torch.randn(B, Tmax, H, hd, device=DEV).bfloat16()
    vc = torch.randn(B, Tmax, H, hd, device=DEV).bfloat16()
    qkv = torch.randn(B, 3 * H * hd, device=DEV).bfloat16()
    ln = torch.tensor([L], dtype=torch.int32, device=DEV)
    kr, vr = kc.clone(), vc.clone()
    C.kv_append(qkv, kc, vc, ln)
    R.kv_append(qkv, kr, vr, ln)
    assert torch.equal(kc, kr) and torch.equal(vc, vr)
    o = C.attn_decode(qkv, kc, vc, ln, 1 / math.sqrt(hd))
    ref = R.attn_decode(qkv.float(), kc.float(), vc.float(), ln.cpu(), 1 / math.sqrt(hd))
    assert _rel(o, ref) < 1e-2
    pos = torch.zeros(B, dtype=torch.int64, device=DEV)
    C.step_advance(ln, pos)
    assert ln.item() == L + 1 and pos.tolist() == [L + 1] * B


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("N,K", [(2304, 768), (768, 2048), (50304, 768), (100, 64), (37, 4096)])
@pytest.mark.parametrize("swiglu", [False, True])
def test_gemv_small_m(C, M, N, K, swiglu):
    """Decode-step projection kernel (gemv16_k, M <= 16 rows as an MFMA A tile, K split over
    waves) against the fp32 oracle, with and without bias and with the fused SwiGLU operand
    (the same bf16 operand as swiglu_fwd: compared exactly through a plain call)."""
    torch.manual_seed(23 + M)
    x = torch.randn(M, 2 * K if swiglu else K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    bias = torch.randn(N, device=DEV)
    assert C.gemv_nt_ok(x, w, swiglu)
    for b in (None, bias):
        y = C.gemv_nt(x, w, b, swiglu)
        ref = R.gemv_nt(x, w, b, swiglu)    # fp32 product of the same bf16 operand
        assert y.shape == (M, N) and y.dtype == torch.bfloat16
        assert _rel(y, ref) < 1e-2, (b is None, _rel(y, ref))
    if swiglu:
        assert torch.equal(C.gemv_nt(C.swiglu_fwd(x), w, bias), C.gemv_nt(x, w, bias, True))
    assert not C.gemv_nt_ok(torch.randn(17, K, device=DEV).bfloat16(), w)   # > 16 rows: caller falls back


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("L", [0, 699, 700])   # 700 = full cache: rotate, append nothing
def test_rope_append_matches_rope_then_append(C, hd, L):
    torch.manual_seed(24)
    B, H, Tmax = 3, 5, 700
    kc = torch.randn(B, Tmax, H, hd, device=DEV).bfloat16()
    vc = torch.randn(B, Tmax, H, hd, device=DEV).bfloat16()
    qkv = torch.randn(B, 3 * H * hd, device=DEV).bfloat16()
    pos = torch.randint(0, 900, (B,), device=DEV)
    tab = R.rope_table(1024, hd, 10000.0).to(DEV)
    ln = torch.tensor([L], dtype=torch.int32, device=DEV)
    a, ka, va = qkv.clone(), kc.clone(), vc.clone()
    C.rope_append(a, pos, tab, ka, va, ln)
    b, kb, vb = qkv.clone(), kc.clone(), vc.clone()
    C.rope_(b, pos, tab, 2 * H, hd, False)
    if L < Tmax:
        C.kv_append(b, kb, vb, ln)
    assert torch.equal(a, b) and torch.equal(ka, kb) and torch.equal(va, vb)


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("n", [8, 4096, 3 * 1024 * 1024 + 8, 25 * 1024 * 1024])
def test_fp8_quantize_matches_oracle(C, fmt, n):
    """fp8 current-scaling quantisation (csrc/kernels/fp8.hip): same bytes and scale as the
    PyTorch oracle (ops/fp8.py: the same fp32 operations), including a non-multiple grid."""
    from distributed_pytorch_from_scratch_amd.ops import fp8 as F8
    torch.manual_seed(26)
    x = (torch.randn(n, device=DEV) * 3).bfloat16()
    q, inv = C.fp8_quant(x, fmt)
    qr, invr = F8.quantize_ref(x, fmt)
    assert q.dtype == qr.dtype and inv.shape == ()
    assert torch.equal(inv, invr)
    assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8))


def test_fp8_gemms_against_oracle(C):
    """fp8 forward (e4m3 x e4m3 + bias) and data-gradient (e5m2 x e4m3) GEMMs: close to the
    bf16 product (quantisation error only) and equal to the fp32 product of the quantised
    operands up to the GEMM's accumulation."""
    from distributed_pytorch_from_scratch_amd.ops import fp8 as F8
    torch.manual_seed(27)
    M, N, K = 4096, 2304, 768
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=DEV)
    fw = F8.Fp8Weight(w)
    y = F8.nt(x, fw, b)
    ref = x.float() @ w.float().t() + b
    assert y.dtype == torch.bfloat16 and _rel(y, ref) < 6e-2
    x8, sx = F8.quantize(x, 0)
    refq = (x8.float() * sx) @ (fw.w8.float() * fw.s).t() + b
    assert _rel(y, refq) < 1e-2
    dy = torch.randn(M, N, device=DEV).bfloat16()
    fw.wt8 = fw.w8.t().contiguous()
    dx = F8.nn(dy, fw)
    refd = dy.float() @ w.float()
    assert dx.shape == (M, K) and _rel(dx, refd) < 1e-1


@pytest.mark.parametrize("M,V,valid,start", [(2048, 6288, 6241, 6288 * 7), (100, 50304, 50257, 0),
                                             (300, 500, 500, 500), (65, 37, 30, 0)])   # unaligned rows
def test_ce_bwd_fused_bias_grad(C, M, V, valid, start):
    torch.manual_seed(16)
    logits = torch.randn(M, V, device=DEV).bfloat16()
    tgt = torch.randint(start, start + valid, (M,), device=DEV)
    lse = torch.logsumexp(logits.float()[:, :valid], -1)
    gs = torch.rand(M, device=DEV)
    out = torch.empty_like(logits)
    db = torch.empty(V, device=DEV)
    C.ce_bwd(logits, tgt, lse, gs, start, valid, out, db)
    rout = torch.empty(M, V, device=DEV)
    rdb = torch.empty(V, device=DEV)
    R.ce_bwd(logits.float(), tgt, lse, gs, start, valid, rout, rdb)
    assert _rel(out, rout) < 1e-2 and _rel(db, rdb) < 1e-3


@pytest.mark.parametrize("M,V,valid", [(4096, 50304, 50257), (777, 32000, 32000), (300, 1000, 997),
                                       (50, 4096 * 13, 4096 * 13), (3, 8, 5), (600, 2048, 100)])
@pytest.mark.parametrize("bias", [True, False])
def test_ce_fused_one_pass(C, M, V, valid, bias):
    """TP-1 CE forward + backward in one pass over the logits (ce_fused_k): the ce_fwd_stats rows
    and the in-place (softmax - onehot) * g (+ column sums) against the fp32 oracle, with ignored
    rows (target -1, g = 0) and a padded vocab tail (valid < V)."""
    torch.manual_seed(17)
    logits = (3 * torch.randn(M, V, device=DEV)).bfloat16()
    tgt = torch.randint(0, valid, (M,), device=DEV)
    tgt[::7] = -1
    gs = (tgt >= 0).float() / max(1, int((tgt >= 0).sum()))
    ref_in = logits.float()
    x = logits.clone()
    db = torch.empty(V, device=DEV) if bias else None
    st = C.ce_fused(x, tgt, gs, 0, valid, db)
    assert st is not None
    rdb = torch.empty(V, device=DEV) if bias else None
    rst = R.ce_fused(ref_in, tgt, gs, 0, valid, rdb)
    lse, rlse = st[:, 0] + torch.log(st[:, 1]), rst[:, 0] + torch.log(rst[:, 1])
    assert torch.allclose(lse, rlse, rtol=0, atol=1e-4)
    assert torch.equal(st[:, 2], rst[:, 2])
    assert _rel(x, ref_in) < 1e-2
    assert x[:, valid:].abs().max().item() == 0 if valid < V else True
    if bias:
        assert _rel(db, rdb) < 1e-3


def test_ce_fused_declines_what_it_cannot_run(C):
    x = torch.randn(4, 13, device=DEV).bfloat16()           # V % 8 != 0: the two-pass path
    t = torch.zeros(4, dtype=torch.long, device=DEV)
    assert C.ce_fused(x, t, torch.ones(4, device=DEV), 0, 13) is None
    x = torch.randn(2, 8 * 512 * 14, device=DEV).bfloat16()   # past 13 slots per thread
    assert C.ce_fused(x, t[:2], torch.ones(2, device=DEV), 0, x.size(1)) is None


@pytest.mark.parametrize("M,N,K0,K1", [(768, 768, 8192, 8192), (1000, 776, 4096, 2048), (2304, 768, 32768, 32768)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_tn2_two_buffer_reduction(C, M, N, K0, K1, accumulate):
    """One split-K launch over a reduction dim split across two buffers (the chunked engines'
    weight gradients) == a0^T b0 + a1^T b1 in fp32 (the split length divides K0)."""
    torch.manual_seed(25)
    a0, a1 = torch.randn(K0, M, device=DEV).bfloat16(), torch.randn(K1, M, device=DEV).bfloat16()
    b0, b1 = torch.randn(K0, N, device=DEV).bfloat16(), torch.randn(K1, N, device=DEV).bfloat16()
    ref = a0.float().t() @ b0.float() + a1.float().t() @ b1.float()
    out = torch.randn(M, N, device=DEV)
    want = out + ref if accumulate else ref
    r = C.gemm_tn2(a0, b0, a1, b1, out, accumulate)
    assert r is not None and r.data_ptr() == out.data_ptr()
    assert _rel(out, want) < 1e-5


@pytest.mark.parametrize("impl,cfg,splits,sched", [(2, -1, 0, -1), (2, 0, 1, 0), (2, 0, 1, 1), (2, 0, 1, 2),
                                                  (2, 0, 1, 3), (2, 0, 1, 4), (2, 1, 1, -1), (2, 0, 3, -1),
                                                  (2, 1, 2, -1), (2, 0, 7, 4), (1, -1, 0, -1),
                                                  (3, -1, 0, -1), (3, 0, 1, 2), (3, 0, 1, 4), (3, 1, 1, -1),
                                                  (3, 0, 3, -1), (3, 1, 2, -1), (3, 0, 7, 4), (3, 1, 5, 2)])
def test_gemm_plans(C, impl, cfg, splits, sched):
    """Every GEMM variant (v3 persistent / v2 / v1, tile configs, K-splits incl. empty
    trailing splits, DMA schedules) on ragged shapes, all three layouts, TN with and without
    accumulate."""
    torch.manual_seed(17)
    M, N, K = 8200, 2104, 712
    a = torch.randn(M, K, device=DEV).bfloat16()
    bt = torch.randn(N, K, device=DEV).bfloat16()
    bn = torch.randn(K, N, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    at = torch.randn(K, M, device=DEV).bfloat16()
    try:
        C.gemm_set_impl(impl)
        C.gemm_force(cfg, splits)
        C.gemm_v2_sched(sched)
        assert _rel(C.gemm_nt(a, bt, bias), R.gemm_nt(a.float(), bt.float(), bias)) < 1e-2
        assert _rel(C.gemm_nn(a, bn), R.gemm_nn(a.float(), bn.float())) < 1e-2
        ref = R.gemm_tn(at.float(), bn.float())
        assert _rel(C.gemm_tn(at, bn), ref) < 1e-2
        acc = torch.randn(M, N, device=DEV)
        want = acc + ref
        C.gemm_tn(at, bn, acc, True)
        assert _rel(acc, want) < 1e-2
    finally:
        C.gemm_set_impl(3)
        C.gemm_force(-1, 0)
        C.gemm_v2_sched(-1)


@pytest.mark.parametrize("with_bias", [True, False])
def test_add_rmsnorm_fwd_fused(C, with_bias):
    torch.manual_seed(18)
    M, D = 777, 768
    y = torch.randn(M, D, device=DEV).bfloat16()
    res = torch.randn(M, D, device=DEV).bfloat16()
    b = torch.randn(D, device=DEV) if with_bias else None
    w = torch.rand(D, device=DEV) + 0.5
    x, h, r = C.add_rmsnorm_fwd(y, b, res, w, 1e-5)
    x2 = C.bias_residual(y, b, res)
    h2, r2 = C.rmsnorm_fwd(x2, w, 1e-5)
    # same math as bias_residual + rmsnorm_fwd (fp32 add order may differ by one bf16 ulp)
    assert (x.float() - x2.float()).abs().max().item() <= 2 ** -7 * x2.float().abs().max().item()
    assert _rel(h, h2) < 1e-2 and torch.allclose(r, r2, rtol=1e-3)
    rx, rh, rr = R.add_rmsnorm_fwd(y.float(), b, res.float(), w, 1e-5)
    assert _rel(h, rh) < 1e-2


def test_rmsnorm_bwd_fused_output_colsum(C):
    torch.manual_seed(19)
    M, D = 1500, 768
    x = torch.randn(M, D, device=DEV).bfloat16()
    w = torch.rand(D, device=DEV) + 0.5
    dy = torch.randn(M, D, device=DEV).bfloat16()
    dres = torch.randn(M, D, device=DEV).bfloat16()
    _, rstd = C.rmsnorm_fwd(x, w, 1e-5)
    db = torch.empty(D, device=DEV)
    dx, dw = C.rmsnorm_bwd(dy, x, w, rstd, dres, db)
    dx2, dw2 = C.rmsnorm_bwd(dy, x, w, rstd, dres)
    assert torch.equal(dx, dx2) and torch.equal(dw, dw2)
    assert _rel(db, dx.float().sum(0)) < 5e-3   # db sums the fp32 values before the bf16 store


def test_fused_adam_fresh_grad_tensors_each_step(C):
    """FusedAdam with new gradient tensors every step (what the training engine returns):
    the table's gradient pointers are patched on the device; trajectory = torch.optim.Adam."""
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    torch.manual_seed(12)
    shapes = [(300, 64), (16384 * 2 + 7,), (4096,)]
    ps = [torch.nn.Parameter(torch.randn(*s, device=DEV)) for s in shapes]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FusedAdam(ps, lr=1e-3, betas=(0.9, 0.95), weight_decay=0.01)
    topt = torch.optim.Adam(ref, lr=1e-3, betas=(0.9, 0.95), weight_decay=0.01)
    keep = []
    for step in range(4):
        gs = [torch.randn_like(p) for p in ps]
        keep.append(gs)                       # distinct live tensors -> distinct pointers
        for p, r, g in zip(ps, ref, gs):
            p.grad, r.grad = g, g.clone()
        opt.step()
        topt.step()
    for p, r in zip(ps, ref):
        assert (p.detach() - r.detach()).abs().max().item() < 1e-5


def test_fused_adam_load_state_dict_after_first_step(C):
    """load_state_dict() after the device table exists swaps in new moment tensors: the next
    step must read the loaded moments (not the freed ones the cached table pointed at)."""
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    torch.manual_seed(13)
    shapes = [(257, 96), (5000,)]
    ps = [torch.nn.Parameter(torch.randn(*s, device=DEV)) for s in shapes]
    donor = [torch.nn.Parameter(torch.randn(*s, device=DEV)) for s in shapes]
    opt = FusedAdam(ps, lr=1e-3)
    dopt = FusedAdam(donor, lr=1e-3)
    for _ in range(3):                         # build opt's table; give the donor other moments
        for p, q in zip(ps, donor):
            p.grad, q.grad = torch.randn_like(p), 5 * torch.randn_like(q)
        opt.step()
        dopt.step()
    import copy
    # deep copies: load_state_dict keeps same-device tensors by reference, and the two
    # optimisers must not share (and double-update) one set of moments
    opt.load_state_dict(copy.deepcopy(dopt.state_dict()))
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    topt = torch.optim.Adam(ref, lr=1e-3)
    topt.load_state_dict(copy.deepcopy(dopt.state_dict()))
    gs = [torch.randn_like(p) for p in ps]
    for p, r, g in zip(ps, ref, gs):
        p.grad, r.grad = g, g.clone()
    opt.step()
    topt.step()
    for p, r in zip(ps, ref):
        assert (p.detach() - r.detach()).abs().max().item() < 1e-5


@pytest.mark.parametrize("backend", ["blas", "lt", "auto"])
def test_gemm_select_tn_and_qkv_rope_paths(C, backend, monkeypatch):
    """gemm_select's hipBLASLt candidates for the fp32 wgrad (incl. accumulate into a live
    gradient) and for the RoPE'd QKV projection match the fp32 oracle; `auto` times both on a
    scratch output, so the live accumulator is updated exactly once."""
    from distributed_pytorch_from_scratch_amd.ops import gemm_select as GS
    monkeypatch.setenv("DPFS_GEMM_BACKEND", backend)
    GS._choice.clear()
    torch.manual_seed(21)
    K_, M_, N_ = 1024, 384, 256
    a = torch.randn(K_, M_, device=DEV).bfloat16()
    b = torch.randn(K_, N_, device=DEV).bfloat16()
    ref = a.float().t() @ b.float()
    c = GS.gemm_tn(C, a, b)
    assert c.dtype == torch.float32 and _rel(c, ref) < 1e-3
    acc = ref.clone()
    GS.gemm_tn(C, a, b, acc, True)
    assert _rel(acc, 2 * ref) < 1e-3
    # QKV + RoPE (2 rotated heads of 64 = q|k, then v)
    Mx, Kx, H, hd = 512, 256, 2, 64
    x = torch.randn(Mx, Kx, device=DEV).bfloat16()
    w = torch.randn(3 * H * hd, Kx, device=DEV).bfloat16() * 0.05
    bias = torch.randn(3 * H * hd, device=DEV) * 0.1
    pos = torch.arange(Mx, device=DEV) % 128
    tab = R.rope_table(256, hd, 10000.0, device=DEV)
    y = GS.gemm_nt_rope(C, x, w, bias, pos, tab, 2 * H, hd)
    yr = R.gemm_nt(x.float(), w.float(), bias, pos, tab, 2 * H, hd)
    assert _rel(y, yr) < 1e-2
    GS._choice.clear()


@pytest.mark.parametrize("layout", [0, 1, 2])
def test_blaslt_direct_every_algorithm(C, layout):
    """hipBLASLt driven through our binding (csrc/blas/blaslt.hip): every heuristic algorithm
    of NT (+ fp32 bias epilogue), NN and TN (fp32 out, overwrite and beta = 1 accumulate) on
    row-major PyTorch operands matches the fp32 oracle."""
    torch.manual_seed(31 + layout)
    M, N, K = 512, 384, 640
    bias = None
    if layout == 0:
        a = torch.randn(M, K, device=DEV).bfloat16()
        b = torch.randn(N, K, device=DEV).bfloat16()
        bias = torch.randn(N, device=DEV)
        ref = a.float() @ b.float().t() + bias
    elif layout == 1:
        a = torch.randn(M, K, device=DEV).bfloat16()
        b = torch.randn(K, N, device=DEV).bfloat16()
        ref = a.float() @ b.float()
    else:
        a = torch.randn(K, M, device=DEV).bfloat16()
        b = torch.randn(K, N, device=DEV).bfloat16()
        ref = a.float().t() @ b.float()
    n = C.lt_algos(layout, M, N, K, bias is not None)
    assert n > 0, "hipBLASLt offered no algorithm"
    for i in range(n):
        out = torch.empty(M, N, device=DEV, dtype=torch.float32 if layout == 2 else torch.bfloat16)
        C.lt_run(layout, a, b, out, bias, i)
        assert _rel(out, ref) < (1e-3 if layout == 2 else 1e-2), f"algorithm {i}"
        if layout == 2:
            C.lt_run(layout, a, b, out, None, i, True)
            assert _rel(out, 2 * ref) < 1e-3, f"algorithm {i} (accumulate)"
    with pytest.raises(RuntimeError):
        C.lt_run(layout, a, b, torch.empty(M + 1, N, device=DEV), bias, 0)


@pytest.mark.parametrize("bn", [0, 256, 192])
@pytest.mark.parametrize("sched", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(8200, 2104, 712), (1000, 776, 2304), (257, 264, 96), (4096, 768, 768),
                                   (520, 1032, 128)])
def test_gemm_v4_bitwise_equals_v3(C, M, N, K, sched, bn):
    """The v4 kernel (one wave per SIMD, 128x128 per wave, 32-deep LDS ring) accumulates every
    output in the same k order as v3, so NT (+bias) and NN results are bit-identical, on both
    DMA streams (K a multiple of 64: descriptor-advancing; else per-lane K checks), at both
    tile widths (256 x 256 and 256 x 192) and on ragged M / N."""
    torch.manual_seed(26)
    a = torch.randn(M, K, device=DEV).bfloat16()
    bt = torch.randn(N, K, device=DEV).bfloat16()
    b_nn = torch.randn(K, N, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    v = {0: 0, 256: 1, 192: 2}[bn]      # per-call variant: v4 at its own / a forced tile width
    try:
        C.gemm4_sched(sched)
        nt4, nn4 = C.gemm_nt(a, bt, bias, variant=v), C.gemm_nn(a, b_nn, variant=v)
        nt3, nn3 = C.gemm_nt(a, bt, bias, variant=3), C.gemm_nn(a, b_nn, variant=3)
    finally:
        C.gemm4_sched(0)
    assert _rel(nt4, R.gemm_nt(a.float(), bt.float(), bias)) < 1e-2
    assert torch.equal(nt4, nt3)
    assert torch.equal(nn4, nn3)


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (2304, 768, 4096), (96, 768, 1000), (776, 2104, 8192)])
@pytest.mark.parametrize("splits", [0, 3])
def test_gemm_v4_tn(C, M, N, K, splits):
    """TN (fp32 weight gradient, split-K slabs) on the v4 kernel, with and without accumulate."""
    torch.manual_seed(27)
    a = torch.randn(K, M, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16()
    try:
        C.gemm_force(-1, splits)
        out = C.gemm_tn(a, b)                       # variant 0: v4 (the default for every layout)
        ref = R.gemm_tn(a.float(), b.float())
        assert _rel(out, ref) < 1e-5
        assert torch.equal(out, C.gemm_tn(a, b, variant=3)) or _rel(C.gemm_tn(a, b, variant=3), ref) < 1e-5
        acc = torch.randn(M, N, device=DEV)
        want = acc + ref
        C.gemm_tn(a, b, acc, True)
        assert _rel(acc, want) < 1e-5
    finally:
        C.gemm_force(-1, 0)


@pytest.mark.parametrize("M,N,K", [(2304, 768, 32768), (768, 2048, 8192), (4096, 768, 4096), (1000, 776, 2048)])
def test_gemm_tn_m32_matches_16x16_form(C, M, N, K):
    """The 32x32x16 TN main loop (default) against the 16x16x32 one and the fp32 oracle, with
    split-K slabs and accumulate (the weight-gradient shapes of GPT-2 small)."""
    torch.manual_seed(31)
    a = torch.randn(K, M, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16()
    ref = R.gemm_tn(a.float(), b.float())
    try:
        C.gemm4_m32(0)
        o16 = C.gemm_tn(a, b)
    finally:
        C.gemm4_m32(1)
    o32 = C.gemm_tn(a, b)
    assert _rel(o32, ref) < 1e-5 and _rel(o16, ref) < 1e-5
    assert _rel(o32, o16) < 1e-5
    acc = torch.randn(M, N, device=DEV)
    want = acc + ref
    C.gemm_tn(a, b, acc, True)
    assert _rel(acc, want) < 1e-5


@pytest.mark.parametrize("layout", ["nn", "nt"])
@pytest.mark.parametrize("M,N,K,splits", [(2048, 768, 50304, 0), (1000, 776, 16384, 3), (520, 1032, 4096, 2)])
def test_gemm_split_k_m32_matches_16x16_form(C, layout, M, N, K, splits):
    """NN / NT with fp32 split-K slabs (the lm_head data gradient's path) on the 32x32x16 main
    loop with K-major operands (the A/B form, gemm4_m32k) against the 16x16x32 loop (default)
    and the fp32 oracle."""
    torch.manual_seed(33)
    a = (torch.randn(M, K, device=DEV) / 16).bfloat16()
    b = (torch.randn(K, N, device=DEV) / 16).bfloat16() if layout == "nn" else \
        (torch.randn(N, K, device=DEV) / 16).bfloat16()
    run = (lambda: C.gemm_nn(a, b)) if layout == "nn" else (lambda: C.gemm_nt(a, b))
    ref = R.gemm_nn(a.float(), b.float()) if layout == "nn" else R.gemm_nt(a.float(), b.float())
    try:
        C.gemm_force(-1, splits)
        C.gemm4_m32k(0)
        o16 = run()
        C.gemm4_m32k(1)
        o32 = run()
    finally:
        C.gemm4_m32k(0)
        C.gemm_force(-1, 0)
    assert _rel(o32, ref) < 1e-2 and _rel(o16, ref) < 1e-2
    assert _rel(o32, o16) < 2e-3


@pytest.mark.parametrize("layout", ["nn", "nt"])
@pytest.mark.parametrize("M,N,K,with_bias", [(4096, 50304, 768, False), (1000, 1032, 512, True), (300, 264, 4096, True)])
def test_gemm_bf16_m32_matches_16x16_form(C, layout, M, N, K, with_bias):
    """NN / NT bf16 output (+ fp32 bias on NT) on 256-wide tiles with the 32x32x16 main loop
    (the A/B form; the lm_head forward's shape first) against the 16x16x32 loop and the oracle,
    ragged M / N included; the non-temporal-store form (variant 5) bit-identical."""
    torch.manual_seed(34)
    a = (torch.randn(M, K, device=DEV) / 8).bfloat16()
    b = (torch.randn(K, N, device=DEV) / 8).bfloat16() if layout == "nn" else \
        (torch.randn(N, K, device=DEV) / 8).bfloat16()
    bias = torch.randn(N, device=DEV) if (with_bias and layout == "nt") else None
    run = (lambda v: C.gemm_nn(a, b, variant=v)) if layout == "nn" else (lambda v: C.gemm_nt(a, b, bias, variant=v))
    ref = R.gemm_nn(a.float(), b.float()) if layout == "nn" else R.gemm_nt(a.float(), b.float(), bias)
    try:
        C.gemm4_m32k(0)
        o16 = run(1)
        C.gemm4_m32k(3)
        o32 = run(1)
        o32nt = run(5)
    finally:
        C.gemm4_m32k(0)
    assert _rel(o32, ref) < 1e-2 and _rel(o16, ref) < 1e-2
    assert _rel(o32, o16) < 2e-3
    assert torch.equal(o32, o32nt)


@pytest.mark.parametrize("layout", ["nt", "nn"])
@pytest.mark.parametrize("K", [768, 4096, 16384])
def test_gemm_stream_k(C, layout, K):
    """The stream-K bf16 kernel (variant 8; 12 = with non-temporal stores) on the N = 768
    projections' shape: 384 tiles of 256 x 256 on 256 CUs, the 128 extra tiles split in K
    halves between two workgroups (fp32 partial hand-off through a flag).  Against the fp32
    oracle and the 256-wide kernel; the 32k x 768 shape is the step's (per-device CU count).
    At a long K (the lm_head data gradient's form) it replaces the split-K slab path."""
    M, N = 32768, 768
    if not C.gemm_sk_applies(M, N, K):
        pytest.skip("stream-K needs 256 x 256 tiles at exactly 1.5 per CU on this device")
    torch.manual_seed(35)
    a = (torch.randn(M, K, device=DEV) / 8).bfloat16()
    b = (torch.randn(N, K, device=DEV) / 8).bfloat16() if layout == "nt" else \
        (torch.randn(K, N, device=DEV) / 8).bfloat16()
    bias = torch.randn(N, device=DEV) if layout == "nt" else None
    run = (lambda v: C.gemm_nt(a, b, bias, variant=v)) if layout == "nt" else (lambda v: C.gemm_nn(a, b, variant=v))
    ref = R.gemm_nt(a.float(), b.float(), bias) if layout == "nt" else R.gemm_nn(a.float(), b.float())
    o = run(8)
    assert _rel(o, ref) < 1e-2 and torch.isfinite(o.float()).all()
    assert _rel(o, run(1)) < 2e-3
    assert torch.equal(run(12), o)
    assert torch.equal(run(8), o)        # (a second launch: the flags are re-zeroed per launch)
    # a column slice of a wider output (the xGMI staging slots' layout)
    if layout == "nt":
        wide = torch.zeros(M, N + 64, device=DEV, dtype=torch.bfloat16)
        C.gemm_nt(a, b, bias, out=wide[:, :N], variant=8)
        assert torch.equal(wide[:, :N], o) and not wide[:, N:].any()
    assert C.gemm_sk_error(False) == 0


def test_gemm_stream_k_starved_producer_raises(C):
    """A stream-K consumer whose producer never raises its flag (test hook) times out after its
    bounded wait; the sticky host-mapped error word then makes the step's error check raise,
    instead of the wrong tile passing silently (gemm4.hip sk_wait)."""
    from distributed_pytorch_from_scratch_amd.ops import _ext
    M, N, K = 32768, 768, 768
    if not C.gemm_sk_applies(M, N, K):
        pytest.skip("stream-K needs 256 x 256 tiles at exactly 1.5 per CU on this device")
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    C.gemm_sk_error(True)
    C.gemm_sk_starve(True)
    C.gemm_nt(a, b, None, variant=8)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="stream-K"):
        _ext.check_device_errors()
    assert C.gemm_sk_error(False) == 0     # reported once, then reset
    C.gemm_nt(a, b, None, variant=8)       # the hook is one-shot: the next launch is clean
    torch.cuda.synchronize()
    assert C.gemm_sk_error(False) == 0


@pytest.mark.parametrize("shapes,K", [([(2304, 768), (768, 768)], 32768), ([(768, 2048), (4096, 768)], 32768),
                                      ([(2304, 768), (768, 768), (4096, 768), (768, 2048)], 8192),
                                      ([(1000, 776), (96, 768), (256, 256)], 2048), ([(384, 768), (768, 128)], 4096)])
def test_gemm_tn_group(C, shapes, K):
    """A layer's weight gradients as ONE grouped 32x32x16 launch (+ one slab reduction) against
    the fp32 oracle, the first GEMM accumulating into an existing gradient."""
    torch.manual_seed(32)
    A = [torch.randn(K, m, device=DEV).bfloat16() for m, _ in shapes]
    B = [torch.randn(K, n, device=DEV).bfloat16() for _, n in shapes]
    outs = [torch.randn(m, n, device=DEV) for m, n in shapes]
    acc = [1] + [0] * (len(shapes) - 1)
    want = [(o.clone() if a_ else 0) + R.gemm_tn(a.float(), b.float()) for o, a, b, a_ in zip(outs, A, B, acc)]
    assert C.gemm_tn_group(A, B, outs, acc)
    for o, w in zip(outs, want):
        assert _rel(o, w) < 1e-5


@pytest.mark.parametrize("shapes,K0,K1", [([(2304, 768), (768, 768)], 16384, 16384),
                                           ([(768, 2048), (4096, 768)], 8192, 8192),
                                           ([(1000, 776), (96, 768), (256, 256)], 2048, 1024),
                                           ([(384, 768), (768, 128)], 4096, 3072)])
def test_gemm_tn_group_two_buffers(C, shapes, K0, K1):
    """A chunked step's weight gradients as ONE grouped launch over both ping-pong chunks' rows
    (the K-split length divides the first buffer's rows; items past it read the second
    buffers) against the fp32 oracle, the first GEMM accumulating."""
    torch.manual_seed(37)
    A = [torch.randn(K0, m, device=DEV).bfloat16() for m, _ in shapes]
    B = [torch.randn(K0, n, device=DEV).bfloat16() for _, n in shapes]
    A2 = [torch.randn(K1, m, device=DEV).bfloat16() for m, _ in shapes]
    B2 = [torch.randn(K1, n, device=DEV).bfloat16() for _, n in shapes]
    outs = [torch.randn(m, n, device=DEV) for m, n in shapes]
    acc = [1] + [0] * (len(shapes) - 1)
    want = [(o.clone() if a_ else 0) + R.gemm_tn(a.float(), b.float()) + R.gemm_tn(a2.float(), b2.float())
            for o, a, b, a2, b2, a_ in zip(outs, A, B, A2, B2, acc)]
    assert C.gemm_tn_group(A, B, outs, acc, A2, B2)
    for o, w in zip(outs, want):
        assert _rel(o, w) < 1e-5


def test_gemm_tn_group_declines(C):
    a = torch.randn(1000, 256, device=DEV).bfloat16()     # K % 64 != 0: not grouped
    outs = [torch.empty(256, 256, device=DEV)] * 2
    assert not C.gemm_tn_group([a, a], [a, a], outs, [0, 0])


def test_gemm_v4_split_k_bf16_long_k(C):
    """bf16-output GEMM with a long K (the lm_head data gradient: N = d_model, K = vocab shard)
    takes the split-K fp32 slab path on v4."""
    torch.manual_seed(28)
    M, N, K = 2048, 768, 50304
    a = (torch.randn(M, K, device=DEV) / 16).bfloat16()
    b = (torch.randn(K, N, device=DEV) / 16).bfloat16()
    out = C.gemm_nn(a, b)
    assert _rel(out, R.gemm_nn(a.float(), b.float())) < 1e-2



@pytest.mark.parametrize("M,K,H,hd", [(4096, 768, 12, 64), (300, 256, 12, 64), (2048, 4096, 32, 128)])
def test_gemm_nt_column_slice_out(C, M, K, H, hd):
    """The packed QKV projection as two launches into one buffer (ops/gemm_select.gemm_nt_rope
    "ours_split"): the rotated Q|K columns (RoPE epilogue) and the V columns written through
    row-strided column slices are bit-identical to the single fused launch (head_dim 64, and 128
    at the LLaMA-7B shape)."""
    torch.manual_seed(46)
    N, rot = 3 * H * hd, 2 * H * hd
    x = (torch.randn(M, K, device=DEV) / 4).bfloat16()
    w = (torch.randn(N, K, device=DEV) / 4).bfloat16()
    b = torch.randn(N, device=DEV)
    pos = torch.arange(M, device=DEV) % 1024
    tab = R.rope_table(1024, hd, 10000.0, device=DEV)
    ref = C.gemm_nt(x, w, b, pos, tab, 2 * H, hd)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C.gemm_nt(x, w[:rot], b[:rot], pos, tab, 2 * H, hd, out=y[:, :rot])
    C.gemm_nt(x, w[rot:], b[rot:], out=y[:, rot:])
    assert torch.equal(y, ref)


@pytest.mark.parametrize("M,F_,K,with_bias", [(4096, 2048, 768, True), (1000, 256, 512, False)])
def test_gemm_nt_swiglu_epilogue(C, M, F_, K, with_bias):
    """Gate|up GEMM with SwiGLU in the epilogue (gemm4.hip SwiOut): the natural [gate | up]
    weight / bias are read with their rows interleaved (reference.gu_perm, no copy), so gu is
    bit-identical to the plain GEMM on an interleaved copy and h to the SwiGLU pass over it, and
    both match the fp32 oracle of the natural layout; the interleaved SwiGLU backward returns the
    natural-layout gradient and bias gradient (oracle)."""
    torch.manual_seed(43)
    x = (torch.randn(M, K, device=DEV) / 4).bfloat16()
    w = (torch.randn(2 * F_, K, device=DEV) / 4).bfloat16()
    b = torch.randn(2 * F_, device=DEV) if with_bias else None
    wp = R.gu_perm(w).contiguous()
    bp = R.gu_perm(b).contiguous() if with_bias else None
    r = C.gemm_nt_swiglu(x, w, b)
    assert len(r) == 2, "fused kernel declined the shape"
    gu, h = r
    assert torch.equal(gu, C.gemm_nt(x, wp, bp))
    assert torch.equal(h, C.swiglu_fwd(gu, True))
    gu_ref = R.gemm_nt(x.float(), w.float(), b)
    assert _rel(R.gu_unperm(gu.float(), 1), gu_ref) < 1e-2
    assert _rel(h.float(), R.swiglu_fwd(gu_ref)) < 2e-2
    dh = torch.randn(M, F_, device=DEV).bfloat16()
    db = torch.empty(2 * F_, device=DEV)
    dgu = C.swiglu_bwd(dh, gu, db, True)
    db_ref = torch.empty(2 * F_, device=DEV)
    dgu_ref = R.swiglu_bwd(dh.float(), R.gu_unperm(gu.float(), 1), db_ref)
    assert _rel(dgu.float(), dgu_ref) < 1e-2
    assert _rel(db, db_ref) < 1e-3
    assert torch.equal(dgu, C.swiglu_bwd(dh, R.gu_unperm(gu, 1).contiguous(), None))


@pytest.mark.parametrize("M,F_,K,perm", [(4096, 2048, 768, True), (1000, 256, 512, True), (777, 320, 64, False),
                                         (300, 2048, 1024, True)])
def test_gemm_nn_swiglu_bwd_epilogue(C, M, F_, K, perm):
    """Down-projection data gradient with the SwiGLU backward in the epilogue (gemm4.hip
    SwiBwd): dgu is bit-identical to gemm_nn followed by the SwiGLU-backward pass (the epilogue
    rounds dy w to bf16 exactly where the separate pass read it), matches the fp32 oracle, and
    the gate|up bias gradient from the kernel's per-wave partials matches the oracle's column
    sums; ragged M (partial row tiles) and a natural-layout gu (perm = False) included."""
    torch.manual_seed(44)
    dy = (torch.randn(M, K, device=DEV) / 4).bfloat16()
    w = (torch.randn(K, F_, device=DEV) / 4).bfloat16()
    gu = torch.randn(M, 2 * F_, device=DEV).bfloat16()
    db = torch.full((2 * F_,), float("nan"), device=DEV)
    r = C.gemm_nn_swiglu_bwd(dy, w, gu, db, perm)
    assert len(r) == 1, "fused kernel declined the shape"
    dgu = r[0]
    ds = C.gemm_nn(dy, w)
    db2 = torch.empty(2 * F_, device=DEV)
    assert torch.equal(dgu, C.swiglu_bwd(ds, gu, db2, perm))
    db_ref = torch.empty(2 * F_, device=DEV)
    gu_nat = R.gu_unperm(gu.float(), 1) if perm else gu.float()
    dgu_ref = R.swiglu_bwd(R.gemm_nn(dy.float(), w.float()), gu_nat, None)
    assert _rel(dgu.float(), dgu_ref) < 1e-2
    # bias grad: the oracle's column sums over the same bf16-rounded dy w the kernel uses
    R.swiglu_bwd(ds.float(), gu_nat, db_ref)
    assert _rel(db, db_ref) < 1e-4 and torch.isfinite(db).all()
    assert _rel(db, db2) < 1e-5
    # without a bias gradient the kernel writes no partials and the same dgu
    assert torch.equal(C.gemm_nn_swiglu_bwd(dy, w, gu, None, perm)[0], dgu)
    # one gate / up row block in flight instead of two (the A/B hook): bit-identical
    try:
        C.gemm4_swb_depth(1)
        db1 = torch.empty(2 * F_, device=DEV)
        assert torch.equal(C.gemm_nn_swiglu_bwd(dy, w, gu, db1, perm)[0], dgu)
        assert torch.equal(db1, db)
    finally:
        C.gemm4_swb_depth(2)


@pytest.mark.parametrize("B,T,H,causal", [(2, 1024, 3, True), (1, 1000, 2, True), (3, 777, 1, True),
                                           (1, 192, 2, True), (1, 64, 1, True), (2, 2048, 1, True),
                                           (1, 1100, 1, True), (2, 256, 2, False), (1, 300, 2, False)])
def test_attention_bwd_dkdv4(C, B, T, H, causal):
    """impl 7: the dQ kernel + the 64-keys-per-wave dK/dV kernel (one wave per SIMD, asm-owned
    AGPR accumulators, K pre-scaled).  Same products in the same order as impl 9 (the v3 pair
    with the K pre-scale): bit-identical to it, incl.
    the inverse RoPE and the QKV bias gradient (32-key partial rows); ragged T (partial 256-key
    blocks, bias rows past the last key), non-causal, strided views; and the fp32 oracle."""
    torch.manual_seed(48)
    hd = 64
    qkv = torch.randn(B * T, 3 * H * hd, device=DEV).bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    o, lse = C.attn_fwd(q, k, v, 0.125, causal)
    do = torch.randn_like(o)
    pos = torch.randint(0, 4096, (B * T,), device=DEV)
    tab = R.rope_table(4096, hd, 10000.0).to(DEV)
    outs = []
    for impl in (7, 9):
        for rope in (False, True):
            d = torch.full_like(qkv, float("nan"))
            dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
            db = torch.full((3 * H * hd,), float("nan"), device=DEV)
            C.attn_bwd(do, q, k, v, o, lse, 0.125, causal, dq, dk, dv, pos if rope else None, tab if rope else None,
                       dbias=db, impl=impl)
            outs.append((d, db))
    for i in range(2):
        assert torch.equal(outs[i][0], outs[2 + i][0]) and torch.equal(outs[i][1], outs[2 + i][1])
    d = outs[0][0]
    assert torch.isfinite(d.float()).all()
    rq, rk, rv = (torch.empty(B, T, H, hd, device=DEV) for _ in range(3))
    R.attn_bwd(do.float(), q.float(), k.float(), v.float(), o.float(), lse, 0.125, causal, rq, rk, rv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    assert _rel(dq, rq) < 3e-2 and _rel(dk, rk) < 3e-2 and _rel(dv, rv) < 3e-2


@pytest.mark.parametrize("M", [1, 1000, 32768, 70001])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_ce_grad_scale(C, M, gdt):
    """The CE backward's per-row loss gradient valid * gloss / n_valid in one launch (device
    scalars, no host sync) against the oracle."""
    torch.manual_seed(49)
    valid = (torch.rand(M, device=DEV) > 0.2).float()
    gloss = torch.tensor(0.37, device=DEV).to(gdt)
    n = valid.sum().clamp_min(1.0)
    acc = torch.stack([torch.tensor(3.0, device=DEV), n])     # n_valid as a view, as the engine passes it
    gs = C.ce_grad_scale(valid, gloss, acc[1])
    assert torch.allclose(gs, R.ce_grad_scale(valid, gloss, acc[1]), rtol=1e-6, atol=0)
