"""HBM planner vs the allocator on an MI355X: the estimated per-rank peak of a steady-state
training step (utils/memory.py) within 10 % of ``torch.cuda.max_memory_allocated`` for GPT-2
small, a 2-layer LLaMA-2-7B slice and a 2-layer 13B slice at seq 8192 (with recompute, as
the planner picks for the whole 13B model on one GPU)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _measure(name, layers, seq, batch, recompute):
    from distributed_pytorch_from_scratch_amd.engine import TrainStep
    from distributed_pytorch_from_scratch_amd.models import Transformer, get_preset
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    from distributed_pytorch_from_scratch_amd.utils import memory as MEM
    kw = dict(recompute=recompute)
    if layers:
        kw["num_layers"] = layers
    args = get_preset(name, **kw)
    dev = torch.device("cuda", 0)
    torch.cuda.empty_cache()
    base = torch.cuda.memory_allocated(dev)
    model = Transformer.from_args(args).to(dev)
    model.reset_parameters()
    opt = FusedAdam(model.parameters(), lr=1e-4)
    step = TrainStep(model, opt)
    g = torch.Generator(device=dev).manual_seed(0)
    ids = torch.randint(0, args.vocab_size, (batch, seq + 1), device=dev, generator=g)
    pos = torch.arange(seq, device=dev).unsqueeze(0).expand(batch, seq).contiguous()
    step(ids[:, :-1], pos, ids[:, 1:])          # first step: kernel choices, optimizer state
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    step(ids[:, :-1], pos, ids[:, 1:])          # steady state (previous grads alive in forward)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated(dev) - base
    est = MEM.estimate(args, MEM.Layout(tp=1, seq=seq, batch=batch, recompute=recompute))
    del model, opt, step
    torch.cuda.empty_cache()
    return peak, est


@pytest.mark.parametrize("name,layers,seq,batch,recompute", [
    ("gpt2-small", None, 1024, 32, False),
    ("llama2-7b", 2, 4096, 2, False),
    ("llama-13b", 2, 8192, 1, True),
])
def test_estimate_within_10_percent_of_measured_peak(name, layers, seq, batch, recompute):
    peak, est = _measure(name, layers, seq, batch, recompute)
    ratio = est.peak / peak
    print(f"{name} L={layers} seq={seq} b={batch} rc={recompute}: measured {peak / 2**30:.2f} GiB, "
          f"estimated {est.gb():.2f} GiB ({est.phase}), ratio {ratio:.3f}\n{est.table()}")
    assert 0.9 <= ratio <= 1.1, (ratio, est.table())
