"""Relayed TP = 2 collectives (parallel/relay.py) on CPU / gloo.

Each TP pair's exchange is split over the direct link and two-hop paths through every other
rank of the WORLD; the results must equal the plain pairwise reduce-scatter / all-gather /
all-reduce for every message size (including sizes too small to relay and odd remainders), on
4 and 8 ranks, and a DP x TP = 2 training step over the relay must follow the RCCL-transport
(gloo here) trajectory.
"""
import os

import pytest
import torch

from dist_helpers import run_distributed


def _collectives(rank, world, sizes):
    os.environ["DPFS_TP_COMM"] = "relay"
    import torch.distributed as dist
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm, tp_comm
    p = pm.get_pgm()
    assert p.tp_size == 2 and p.dp_size == world // 2
    errs = []
    for n in sizes:                     # n = elements of the full (pair-summed) tensor
        g = torch.Generator().manual_seed(1000 * n + rank)
        x = torch.randn(n, generator=g)
        # oracle: the pair's sum via all_reduce on the TP group
        ref = x.clone()
        dist.all_reduce(ref, group=p.tp_group)
        out = torch.empty(n // 2)
        h = tp_comm.reduce_scatter(out, x, async_op=True)
        if h is not None:
            h.wait()
        errs.append((out - ref.view(2, -1)[p.tp_rank]).abs().max().item())
        full = torch.empty(n)
        h = tp_comm.all_gather(full, out, async_op=True)
        if h is not None:
            h.wait()
        errs.append((full - ref).abs().max().item())
        y = x.clone()
        h = tp_comm.all_reduce(y, async_op=True)
        if h is not None:
            h.wait()
        errs.append((y - ref).abs().max().item())
    info = tp_comm.info()
    return max(errs), info["transport"] if info else None


@pytest.mark.parametrize("world", [4, 8])
def test_relay_collectives_match_pairwise(world):
    sizes = [16, 48, 1000, 4096 + 40, 100_000]   # tiny (direct only), ragged units, large
    res = run_distributed(_collectives, world, sizes, tp_size=2)
    for r, (err, transport) in res.items():
        assert err < 1e-5, (r, err)
        assert transport == "/".join(f"{op}:s=relay,m=relay,l=relay" for op in ("all_reduce", "reduce_scatter", "all_gather"))


def _train(rank, world, transport, sp):
    os.environ["DPFS_TP_COMM"] = transport
    import torch.distributed as dist
    from distributed_pytorch_from_scratch_amd.engine import TrainStep
    from distributed_pytorch_from_scratch_amd.models import ModelArgs, Transformer
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    p = pm.get_pgm()
    m = Transformer.from_args(ModelArgs(attn_dim=64, ffn_dim=128, num_heads=4, num_layers=2, vocab_size=96,
                                        maxlen=32, vocab_pad_to=1, sequence_parallel=sp))
    set_seed(0)
    m.reset_parameters()
    step = TrainStep(m, torch.optim.Adam(m.parameters(), lr=1e-3))
    losses = []
    for s in range(3):
        g = torch.Generator().manual_seed(50 + s)
        ids = torch.randint(0, 96, (8, 16), generator=g)
        tgt = torch.randint(0, 96, (8, 16), generator=g)
        pos = torch.arange(16).repeat(8, 1)
        sl = slice(2 * p.dp_rank, 2 * p.dp_rank + 2)
        loss = step(ids[sl], pos[sl], tgt[sl]).reshape(1)
        dist.all_reduce(loss, group=p.dp_group)
        losses.append(loss.item() / p.dp_size)
    return losses


@pytest.mark.parametrize("sp", [True, False])
def test_relay_training_step_matches(sp):
    """DP 2 x TP 2 (4 ranks): the fused engine (SP: reduce-scatter / all-gather; no SP:
    all-reduce) over the relay transport follows the same losses as over torch.distributed."""
    ref = run_distributed(_train, 4, "rccl", sp, tp_size=2)
    got = run_distributed(_train, 4, "relay", sp, tp_size=2)
    for r in range(4):
        assert all(abs(a - b) < 1e-5 for a, b in zip(got[r], ref[r])), (r, got[r], ref[r])


def _ragged(rank, world, base_sizes):
    """Every TP pair passes a DIFFERENT message size in the same collective (real-data batches
    padded per batch on each DP rank): the relay must agree on one unit size over the WORLD."""
    os.environ["DPFS_TP_COMM"] = "relay"
    import torch.distributed as dist
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm, tp_comm
    p = pm.get_pgm()
    errs = []
    for base in base_sizes:
        n = base + 24 * p.dp_rank                 # pair-dependent, even
        g = torch.Generator().manual_seed(7 * n + rank)
        x = torch.randn(n, generator=g)
        ref = x.clone()
        dist.all_reduce(ref, group=p.tp_group)
        out = torch.empty(n // 2)
        h = tp_comm.reduce_scatter(out, x, async_op=True)
        if h is not None:
            h.wait()
        errs.append((out - ref.view(2, -1)[p.tp_rank]).abs().max().item())
        full = torch.empty(n)
        h = tp_comm.all_gather(full, out, async_op=True)
        if h is not None:
            h.wait()
        errs.append((full - ref).abs().max().item())
        for odd in (n + 1, n + 3):                # odd all-reduce counts (zero-padded inside)
            y = torch.randn(odd, generator=g)
            r2 = y.clone()
            dist.all_reduce(r2, group=p.tp_group)
            h = tp_comm.all_reduce(y, async_op=True)
            if h is not None:
                h.wait()
            errs.append((y - r2).abs().max().item())
    return max(errs)


@pytest.mark.parametrize("world", [4, 8])
def test_relay_ragged_sizes_across_pairs(world):
    res = run_distributed(_ragged, world, [48, 1000, 20_000], tp_size=2)
    for r, err in res.items():
        assert err < 1e-5, (r, err)
