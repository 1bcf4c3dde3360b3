"""Multi-rank runs of the fused engine on the real HIP kernels (one MI355X, several ranks).

RCCL refuses two ranks on one device, so these tests drive the collectives with gloo over
device tensors. That covers everything except the transport: the ping-pong chunk schedule
with async all-reduces, uneven head and vocab shards, the in-engine DP averaging and the
fused Adam step. The TP = k and DP x TP loss trajectories must follow the single-rank one.
The 8-rank RCCL run itself is the driver's scaling bench.
"""
import pytest
import torch

from dist_helpers import run_distributed

pytestmark = pytest.mark.gpu

STEPS = 3


def _train(rank, world, tp, dp, heads, dev="cuda", sp=False, recompute=False, transport=None):
    import os
    if transport:
        os.environ["DPFS_TP_COMM"] = transport
    import torch.distributed as dist
    if dev == "cuda":
        torch.cuda.set_device(0)
    from distributed_pytorch_from_scratch_amd.models import get_preset, Transformer
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    from distributed_pytorch_from_scratch_amd.engine import TrainStep
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    args = get_preset("gpt2-small", num_layers=2, num_heads=heads, vocab_size=1000, vocab_pad_to=1,
                      sequence_parallel=sp, recompute=recompute)
    m = Transformer.from_args(args).to(dev)
    set_seed(0)
    m.reset_parameters()
    assert m.fused_supported()
    opt = FusedAdam(m.parameters(), lr=1e-3)
    step = TrainStep(m, opt)
    p = pm.pgm
    B, T = 4, 256
    losses = []
    for s in range(STEPS):
        g = torch.Generator().manual_seed(100)   # same batch: the loss must fall
        ids = torch.randint(0, args.vocab_size, (B, T), generator=g)
        tgt = torch.randint(0, args.vocab_size, (B, T), generator=g)
        pos = torch.arange(T).repeat(B, 1)
        sl = slice(p.dp_rank * B // dp, (p.dp_rank + 1) * B // dp)
        loss = step(ids[sl].to(dev), pos[sl].to(dev), tgt[sl].to(dev)).float()
        if dp > 1:
            dist.all_reduce(loss, group=p.dp_group)
            loss /= dp
        losses.append(loss.item())
    if dev == "cuda":
        torch.cuda.synchronize()
    return losses


def _ref(heads):
    return run_distributed(_train, 1, 1, 1, heads, tp_size=1)[0]


@pytest.mark.parametrize("world,tp,dp,heads,sp", [(2, 2, 1, 12, False), (4, 4, 1, 6, False), (4, 2, 2, 12, False),
                                                 (2, 2, 1, 12, True), (4, 2, 2, 12, True)])
def test_multirank_engine_follows_single_rank(world, tp, dp, heads, sp):
    ref = _ref(heads)
    res = run_distributed(_train, world, tp, dp, heads, "cuda", sp, tp_size=tp)
    for r, losses in res.items():
        for a, b in zip(losses, ref):
            assert abs(a - b) < 2e-2 * max(1.0, abs(b)), (r, losses, ref)
    # training moves the loss, identically on every rank
    assert ref[-1] < ref[0]
    assert len({tuple(v) for v in res.values()}) == 1


@pytest.mark.parametrize("sp", [True, False])
def test_relay_transport_engine_follows_single_rank(sp):
    """DP 2 x TP 2 on the GPU kernels with the TP collectives relayed through the other pair
    (parallel/relay.py; gloo point-to-point here, fenced, RCCL on a real node)."""
    ref = _ref(12)
    res = run_distributed(_train, 4, 2, 2, 12, "cuda", sp, False, "relay", tp_size=2)
    for r, losses in res.items():
        for a, b in zip(losses, ref):
            assert abs(a - b) < 2e-2 * max(1.0, abs(b)), (r, losses, ref)
    assert len({tuple(v) for v in res.values()}) == 1
