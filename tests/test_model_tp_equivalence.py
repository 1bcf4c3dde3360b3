"""TP is numerically transparent (SURVEY.md §0 key invariant), CPU/gloo.

Same seed => TP=k weights equal the TP=1 / vanilla weights exactly, and the loss trajectory
over several Adam steps matches to ~1e-5 (fp32).  Also covers uneven head partitions (6
heads over 4 ranks), a non-divisible vocab, sequence parallelism and the reference
state-dict layout.
"""
import pytest
import torch
import torch.nn.functional as F

from dist_helpers import run_distributed
from vanilla_model import VanillaTransformer


def _batch(V, B, T, seed=123):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (B, T), generator=g)
    tgt = torch.randint(0, V, (B, T), generator=g)
    tgt[0, -3:] = -1  # ignored positions
    pos = torch.arange(T).unsqueeze(0).repeat(B, 1)
    return ids, pos, tgt


CFG = dict(attn_dim=64, ffn_dim=128, num_heads=4, num_layers=2, vocab_size=96, maxlen=64)


def _train_parallel(rank, world, cfg, steps, sp, use_loss_api, fused=True):
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    args = ModelArgs(**cfg, vocab_pad_to=1, sequence_parallel=sp)
    m = Transformer.from_args(args)
    m.use_fused_engine = fused
    set_seed(0)
    m.reset_parameters()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for s in range(steps):
        ids, pos, tgt = _batch(cfg["vocab_size"], 2, 16, seed=100 + s)
        if use_loss_api:
            loss = m.loss(ids, pos, tgt)
        else:
            logits = m(ids, pos)
            loss = F.cross_entropy(logits.reshape(-1, logits.size(-1)), tgt.reshape(-1), ignore_index=-1)
        opt.zero_grad()
        loss.backward()
        if sp:
            from distributed_pytorch_from_scratch_amd.parallel.grad_sync import allreduce_sequence_parallel_grads
            allreduce_sequence_parallel_grads(m)
        opt.step()
        losses.append(loss.item())
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    return losses, sd


def _train_vanilla(cfg, steps):
    m = VanillaTransformer(**cfg)
    torch.manual_seed(0)      # RNG replay: same state right before reset_parameters()
    m.reset_parameters()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for s in range(steps):
        ids, pos, tgt = _batch(cfg["vocab_size"], 2, 16, seed=100 + s)
        logits = m(ids, pos)
        loss = F.cross_entropy(logits.reshape(-1, logits.size(-1)), tgt.reshape(-1), ignore_index=-1)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses, m


@pytest.mark.parametrize("world", [1, 2, 4])
def test_tp_matches_vanilla_loss_trajectory(world):
    van, _ = _train_vanilla(CFG, 3)
    res = run_distributed(_train_parallel, world, CFG, 3, False, True)
    for r in range(world):
        assert torch.allclose(torch.tensor(res[r][0]), torch.tensor(van), atol=2e-5), (res[r][0], van)


def test_tp_gathered_logits_api_matches():
    van, _ = _train_vanilla(CFG, 2)
    res = run_distributed(_train_parallel, 2, CFG, 2, False, False)
    assert torch.allclose(torch.tensor(res[0][0]), torch.tensor(van), atol=2e-5)


def test_uneven_heads_and_vocab():
    cfg = dict(CFG, num_heads=8, attn_dim=48, vocab_size=97)   # 8 heads of 6 over 3 ranks
    van, _ = _train_vanilla(cfg, 2)
    res = run_distributed(_train_parallel, 3, cfg, 2, False, True)
    for r in range(3):
        assert torch.allclose(torch.tensor(res[r][0]), torch.tensor(van), atol=2e-5)


@pytest.mark.parametrize("world,fused", [(2, True), (4, True), (2, False)])
def test_sequence_parallel_matches(world, fused):
    """SP through the fused SP engine (models/fused_engine_sp.py) and through the modular
    layers: same loss trajectory as the vanilla model, replicated params identical on every
    rank after the steps."""
    van, _ = _train_vanilla(CFG, 3)
    res = run_distributed(_train_parallel, world, CFG, 3, True, True, fused)
    for r in range(world):
        assert torch.allclose(torch.tensor(res[r][0]), torch.tensor(van), atol=2e-5), (res[r][0], van)
    for key in ("layers.0.norm1.scale", "layers.1.attn.wo.bias", "layers.1.ffn.down_proj.bias", "norm.scale"):
        for r in range(1, world):
            assert torch.equal(res[r][1][key], res[0][1][key]), key


@pytest.mark.parametrize("world,sp", [(1, False), (2, False), (2, True)])
def test_activation_recompute_matches(world, sp):
    """ModelArgs.recompute: the engines keep only each layer's input and re-run the layer
    forward (collectives included) in backward -- same trajectory as the vanilla model."""
    cfg = dict(CFG, recompute=True)
    van, _ = _train_vanilla(CFG, 3)
    res = run_distributed(_train_parallel, world, cfg, 3, sp, True, True)
    for r in range(world):
        assert torch.allclose(torch.tensor(res[r][0]), torch.tensor(van), atol=2e-5), (res[r][0], van)


def test_state_dict_layout_is_reference_layout():
    cfg = dict(CFG)
    res = run_distributed(_train_parallel, 2, cfg, 1, False, True)
    sd = res[0][1]
    L = cfg["num_layers"]
    assert len(sd) == 1 + L * 16 + 1 + 2  # emb, 16 per layer, norm, lm_head w+b (196 at L=12)
    d, f, V = cfg["attn_dim"], cfg["ffn_dim"], cfg["vocab_size"]
    assert sd["layers.0.attn.wq.weight"].shape == (d // 2, d)
    assert sd["layers.0.attn.wo.weight"].shape == (d, d // 2)
    assert sd["layers.0.attn.wo.bias"].shape == (d,)
    assert sd["layers.0.ffn.gate_proj.weight"].shape == (f // 2, d)
    assert sd["layers.0.ffn.down_proj.weight"].shape == (d, f // 2)
    assert sd["embedding.weight"].shape == (V // 2, d)
    assert sd["lm_head.bias"].shape == (V // 2,)
    assert "layers.1.norm2.scale" in sd and "norm.scale" in sd


def _load_roundtrip(rank, world):
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    set_seed(0)
    m = Transformer.from_args(ModelArgs(**CFG, vocab_pad_to=1))
    m.reset_parameters()
    sd = m.state_dict()
    set_seed(1)
    m2 = Transformer.from_args(ModelArgs(**CFG, vocab_pad_to=1))
    m2.reset_parameters()
    m2.load_state_dict(sd)
    ids, pos, tgt = _batch(CFG["vocab_size"], 2, 8)
    return (m(ids, pos) - m2(ids, pos)).abs().max().item()


def test_state_dict_roundtrip():
    res = run_distributed(_load_roundtrip, 2)
    assert res[0] == 0.0 and res[1] == 0.0


def _grads_chunked(rank, world, cfg, sp, chunks):
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    m = Transformer.from_args(ModelArgs(**cfg, vocab_pad_to=1, sequence_parallel=sp))
    set_seed(0)
    m.reset_parameters()
    m.chunks = chunks
    ids, pos, tgt = _batch(cfg["vocab_size"], 4, 16, seed=7)
    loss = m.loss(ids, pos, tgt)
    loss.backward()
    if sp:
        from distributed_pytorch_from_scratch_amd.parallel.grad_sync import allreduce_sequence_parallel_grads
        allreduce_sequence_parallel_grads(m)
    return loss.item(), {n: p.grad.clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("sp", [False, True])
def test_chunk_counts_give_same_grads(sp):
    """The chunked engines sum each weight gradient over the ping-pong chunks two at a time
    (ops.gemm_select.gemm_tn_pair) plus a leftover single chunk: 1, 2, 3 and 4 chunks of a
    4-sequence batch give the same loss and gradients at TP 2."""
    res = {c: run_distributed(_grads_chunked, 2, CFG, sp, c)[0] for c in (1, 2, 3, 4)}
    for c in (2, 3, 4):
        assert abs(res[c][0] - res[1][0]) < 1e-5
        for n, g in res[1][1].items():
            assert torch.allclose(res[c][1][n], g, atol=1e-5, rtol=1e-4), (c, n)


@pytest.mark.parametrize("world,sp,recompute", [(1, False, False), (2, False, True), (2, True, False)])
def test_swiglu_epilogue_layout_matches(world, sp, recompute, monkeypatch):
    """The layout of the fused gate|up + SwiGLU GEMM epilogue (ops.reference.gu_perm: weight
    rows, bias and gate|up activations interleaved in 64-blocks; the weight gradient
    un-interleaved once per layer and step), run through the CPU oracle with
    ModelArgs.swiglu_epilogue=True in both engines (and the recompute path): the same loss
    trajectory and parameters as the natural layout."""
    cfg = dict(CFG, recompute=recompute)
    base = run_distributed(_train_parallel, world, dict(cfg, swiglu_epilogue=False), 3, sp, True, True)
    fused = run_distributed(_train_parallel, world, dict(cfg, swiglu_epilogue=True), 3, sp, True, True)
    for r in range(world):
        assert torch.allclose(torch.tensor(fused[r][0]), torch.tensor(base[r][0]), atol=1e-6), (fused[r][0], base[r][0])
        for key, v in base[r][1].items():
            assert torch.allclose(fused[r][1][key], v, atol=1e-5), key
