"""Autograd collectives and the vocab-parallel cross-entropy (CPU / gloo)."""
import pytest
import torch
import torch.nn.functional as F

from dist_helpers import run_distributed


def _comm(rank, world):
    from distributed_pytorch_from_scratch_amd.parallel import Split, Reduce, Copy, Gather, ScatterSeq, GatherSeq
    torch.manual_seed(0)
    full = torch.randn(4, 6 * world, requires_grad=True)       # same on every rank
    # Split fwd = my slice; bwd = all-gather of slices
    y = Split.apply(full)
    assert torch.equal(y, full[:, rank * 6:(rank + 1) * 6])
    (y * (rank + 1)).sum().backward()
    expect = torch.cat([torch.full((4, 6), float(r + 1)) for r in range(world)], 1)
    assert torch.equal(full.grad, expect)
    # Reduce fwd = sum over ranks; bwd identity
    x = torch.full((3,), float(rank + 1), requires_grad=True)
    out = Reduce.apply(x * 1.0)
    assert torch.allclose(out, torch.full((3,), world * (world + 1) / 2))
    # Copy fwd identity; bwd all-reduce
    c = torch.ones(3, requires_grad=True)
    (Copy.apply(c) * (rank + 1)).sum().backward()
    assert torch.allclose(c.grad, torch.full((3,), world * (world + 1) / 2))
    # Gather fwd = concat; bwd = my slice
    g = torch.full((2, 3), float(rank), requires_grad=True)
    go = Gather.apply(g)
    assert go.shape == (2, 3 * world) and torch.equal(go[:, 3 * rank:3 * rank + 3], g.detach())
    go.sum().backward()
    assert torch.equal(g.grad, torch.ones(2, 3))
    # uneven Gather (sizes)
    sizes = [2 + r for r in range(world)]
    u = torch.full((2, sizes[rank]), float(rank), requires_grad=True)
    uo = Gather.apply(u, sizes)
    assert uo.shape == (2, sum(sizes))
    # sequence-parallel pair: scatter(sum) then gather
    s = torch.arange(world * 2 * 3, dtype=torch.float32).view(world * 2, 3) * (rank + 1)
    sc = ScatterSeq.apply(s.clone().requires_grad_(True))
    tot = torch.arange(world * 2 * 3, dtype=torch.float32).view(world * 2, 3) * (world * (world + 1) / 2)
    assert torch.allclose(sc, tot[2 * rank:2 * rank + 2])
    ga = GatherSeq.apply(sc)
    assert torch.allclose(ga, tot)
    return True


@pytest.mark.parametrize("world", [2, 3])
def test_comm_ops(world):
    assert all(run_distributed(_comm, world).values())


def _ce(rank, world, V, valid_V, pad_ignore):
    from distributed_pytorch_from_scratch_amd.parallel.cross_entropy import vocab_parallel_cross_entropy
    torch.manual_seed(1)
    M = 17
    full = torch.randn(M, V)
    tgt = torch.randint(0, valid_V, (M,))
    if pad_ignore:
        tgt[3] = -1
    per = V // world
    st = rank * per
    shard = full[:, st:st + per].clone().requires_grad_(True)
    valid = max(0, min(valid_V - st, per))
    loss = vocab_parallel_cross_entropy(shard, tgt, st, valid, inplace_backward=False)
    loss.backward()
    ref_logits = full[:, :valid_V].clone().requires_grad_(True)
    ref = F.cross_entropy(ref_logits, tgt, ignore_index=-1)
    ref.backward()
    ref_grad = torch.zeros(M, V)
    ref_grad[:, :valid_V] = ref_logits.grad
    assert torch.allclose(loss, ref, atol=1e-5)
    assert torch.allclose(shard.grad, ref_grad[:, st:st + per], atol=1e-6)
    return loss.item()


@pytest.mark.parametrize("world,V,valid,ign", [(2, 40, 40, False), (4, 64, 57, True), (1, 32, 30, True)])
def test_vocab_parallel_ce(world, V, valid, ign):
    run_distributed(_ce, world, V, valid, ign)


def _dp(rank, world, fused):
    """DP=2 x TP=2 grid: DP gradient averaging gives the same step as the full batch on one
    replica; the TP groups are {0,1} and {2,3}.  ``fused``: the engine averages inside its
    backward (overlapped) and the hooks stand down; else the bucketed hooks do it."""
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm
    from distributed_pytorch_from_scratch_amd.parallel.grad_sync import DataParallelGradSync
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    p = pm.get_pgm()
    assert (p.dp_size, p.tp_size) == (2, 2) and p.tp_ranks == [2 * p.dp_rank, 2 * p.dp_rank + 1]
    args = ModelArgs(attn_dim=32, ffn_dim=64, num_heads=4, num_layers=1, vocab_size=64, maxlen=16, vocab_pad_to=1)
    m = Transformer.from_args(args)
    m.use_fused_engine = fused
    set_seed(0)
    m.reset_parameters()
    sync = DataParallelGradSync(m, bucket_mb=0.01)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 64, (4, 8), generator=g)
    tgt = torch.randint(0, 64, (4, 8), generator=g)
    pos = torch.arange(8).repeat(4, 1)
    half = slice(2 * p.dp_rank, 2 * p.dp_rank + 2)
    loss = m.loss(ids[half], pos[half], tgt[half])
    loss.backward()
    sync.finish()
    got = {n: q.grad.clone() for n, q in m.named_parameters()}
    m.zero_grad()
    m.loss(ids, pos, tgt).backward()
    sync.finish()
    return max((got[n] - q.grad).abs().max().item() for n, q in m.named_parameters())


@pytest.mark.parametrize("fused", [True, False])
def test_data_parallel_grad_sync(fused):
    res = run_distributed(_dp, 4, fused, tp_size=2)
    assert max(res.values()) < 1e-6


@pytest.mark.parametrize("chunks", [1, 2])
def test_unit_grad_ce_in_forward_matches_two_pass(chunks):
    """TP 1 with ``loss(..., unit_grad=True)`` (engine.TrainStep): the engine writes d logits in
    the forward's single pass over the logits (k.ce_fused); loss and every gradient equal the
    two-pass CE (statistics in forward, d logits in backward), ignored targets included."""
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    args = ModelArgs(attn_dim=32, ffn_dim=64, num_heads=4, num_layers=2, vocab_size=61, maxlen=16)
    m = Transformer.from_args(args)
    m.chunks = chunks
    set_seed(0)
    m.reset_parameters()
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 61, (4, 16), generator=g)
    tgt = torch.randint(0, 61, (4, 16), generator=g)
    tgt[1, 3:9] = -1
    pos = torch.arange(16).repeat(4, 1)
    out = []
    for unit in (False, True):
        m.zero_grad(set_to_none=True)
        loss = m.loss(ids, pos, tgt, unit_grad=unit)
        loss.backward()
        out.append((loss.item(), {n: q.grad.clone() for n, q in m.named_parameters()}))
    (l0, g0), (l1, g1) = out
    assert abs(l0 - l1) < 1e-6
    for n in g0:
        assert torch.allclose(g0[n], g1[n], rtol=1e-5, atol=1e-7), n
