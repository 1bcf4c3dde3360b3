"""The ``auto`` transport decision of parallel/tp_comm.py, exercised without RCCL.

On a real node ``auto`` validates every candidate transport (xGMI kernels, the relayed TP = 2
exchange) against an fp32 process-group sum, times them against the process group, picks a
grid per op and reduces every input of the decision over the TP group (or over the WORLD when
the relay is a candidate), so that every rank takes the same transport for every op.  A rank
that decided differently would issue a different collective sequence and hang its group, so
this is what the first 8-GPU run depends on.  ``DPFS_TP_COMM_AUTO_ANY_BACKEND=1`` runs the
same decision over gloo: on the CPU (relay candidate only) and, marked gpu, with several ranks
sharing one MI355X (xGMI kernels + relay).  The decision is per op AND per message-size class
(``tp_comm.SIZE_CLASSES``: <= 1 MiB, <= 16 MiB, larger), so every case drives messages of all
three classes through the collectives after the decision.  Each case checks: identical
decisions (transport and xGMI grid per op and class) on every rank, the collectives' results
against fp32 sums, and the decision record (``tp_comm.info``) the bench line reports.
"""
import os

import pytest
import torch

from dist_helpers import run_distributed


def _decide(rank, world, dev, sizes):
    os.environ["DPFS_TP_COMM"] = "auto"
    os.environ["DPFS_TP_COMM_AUTO_ANY_BACKEND"] = "1"
    os.environ["DPFS_QUIET"] = "1"
    import torch.distributed as dist
    if dev == "cuda":
        torch.cuda.set_device(0)
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm, tp_comm
    tp_comm.set_fixed_shapes(True)
    p = pm.get_pgm()
    W = p.tp_size
    errs = []
    trace = []
    if dev == "cuda":    # per-rank record of every xGMI launch (op, elements, grid) for diagnosis
        from distributed_pytorch_from_scratch_amd.parallel import xgmi as X
        orig = X.XgmiComm._launch

        def traced(self, op, x, out, timeout_s=None, slot=-1):
            trace.append((op, x.numel(), self._blocks if self.op_blocks[X._NAMES[op]] is None
                          else self.op_blocks[X._NAMES[op]]))
            return orig(self, op, x, out, timeout_s, slot)
        X.XgmiComm._launch = traced
    for i, n in enumerate(sizes):            # the first call decides, the others reuse it
        g = torch.Generator().manual_seed(77 * i + rank)
        x = torch.randn(n, generator=g).to(torch.bfloat16 if dev == "cuda" else torch.float32).to(dev)
        ref = x.float().clone()
        dist.all_reduce(ref, group=p.tp_group)
        part = torch.empty(n // W, dtype=x.dtype, device=dev)
        h = tp_comm.reduce_scatter(part, x, async_op=True)
        if h is not None:
            h.wait()
        full = torch.empty(n, dtype=x.dtype, device=dev)
        h = tp_comm.all_gather(full, part, async_op=True)
        if h is not None:
            h.wait()
        y = x.clone()
        h = tp_comm.all_reduce(y, async_op=True)
        if h is not None:
            h.wait()
        if dev == "cuda":
            torch.cuda.synchronize()
        errs += [(part.float() - ref.view(W, -1)[p.tp_rank]).abs().max().item(),
                 (full.float() - ref).abs().max().item(), (y.float() - ref).abs().max().item()]
    ch = tp_comm._decisions.get(id(p.tp_group))
    xerr = ch.xgmi.error() if ch is not None and ch.xgmi is not None else 0
    anyerr = torch.tensor([float(xerr)])
    dist.all_reduce(anyerr, op=dist.ReduceOp.MAX)
    info = tp_comm.info()
    dec = tp_comm.decision()
    if anyerr.item() == 0:
        tp_comm.reset()
    return dict(err=max(errs), scale=ref.abs().max().item(), dec=dec, info=info, tp_rank=p.tp_rank,
                dp_rank=p.dp_rank, xerr=xerr, trace=trace)


def _check_same(res, tp):
    traces = {r: v["trace"] for r, v in res.items()}
    if any(v["xerr"] for v in res.values()):     # name the first launch where the ranks diverge
        t0 = traces[0]
        div = [(r, next((i for i, (a, b) in enumerate(zip(t0, t)) if a != b), None), len(t))
               for r, t in traces.items()]
        raise AssertionError(f"xGMI timeout on ranks {[r for r, v in res.items() if v['xerr']]}; "
                             f"launches per rank / first divergence from rank 0: {div}; "
                             f"rank 0 tail {t0[-6:]}")
    decs = {r: v["dec"] for r, v in res.items()}
    first = next(iter(decs.values()))
    assert first is not None
    for r, d in decs.items():
        assert d == first, (r, d, first)        # every rank: same transport and grid per op
    for r, v in res.items():
        assert v["err"] <= 2e-2 * max(1.0, v["scale"]), (r, v["err"])
        assert v["info"] is not None and set(v["info"]) >= {"all_reduce", "reduce_scatter", "all_gather",
                                                            "transport"}


# fp32 on the CPU: 16 KiB, 4 MiB, 20 MiB -> classes s, m, l (the first call decides)
CPU_SIZES = [4096, 1 << 20, 5 << 20]


@pytest.mark.parametrize("world", [4, 8])
def test_auto_decision_relay_candidate_cpu(world):
    """tp2 x dp(world/2) on the CPU: the relay is the one candidate; its validation and timing
    are reduced over the WORLD, so every pair takes the same decision per size class."""
    res = run_distributed(_decide, world, "cpu", CPU_SIZES, tp_size=2)
    _check_same(res, 2)
    for v in res.values():
        for c in ("s", "m", "l"):
            assert "relay_ms" in v["info"]["all_reduce"][c] and "rccl_ms" in v["info"]["all_reduce"][c]
        assert "s=" in v["info"]["transport"] and "l=" in v["info"]["transport"]


def test_auto_decision_without_candidates_cpu():
    """Pure TP 4 on the CPU: no candidate transport, the process group carries everything."""
    res = run_distributed(_decide, 4, "cpu", CPU_SIZES[:2], tp_size=4)
    for v in res.values():
        assert set(v["dec"]["use"].values()) == {"rccl"} and len(v["dec"]["use"]) == 9
        assert v["dec"]["op_blocks"] is None
        assert v["err"] < 1e-4


def test_size_classes():
    from distributed_pytorch_from_scratch_amd.parallel import tp_comm
    assert [tp_comm.size_class(b) for b in (1, 1 << 20, (1 << 20) + 16, 16 << 20, (16 << 20) + 16)] == \
        ["s", "s", "m", "m", "l"]


@pytest.mark.gpu
@pytest.mark.parametrize("world,tp", [(2, 2), (4, 2), (4, 4), (8, 8)])
def test_auto_decision_on_one_gpu(world, tp):
    """Several ranks on one MI355X over gloo: the xGMI kernels (two-shot at every grid width,
    the one-shot all-reduce for the small / medium classes) and the relay (tp = 2 with other
    pairs) are validated and timed per size class; every rank must reach the same transport and
    xGMI grid per op and class (8 ranks at tp 8 is the driver's pure-TP layout)."""
    sizes = [8 * tp * 4096, 2 << 20, 12 << 20]     # bf16: classes s, m, l
    res = run_distributed(_decide, world, "cuda", sizes, tp_size=tp)
    _check_same(res, tp)
    for v in res.values():
        ar = v["info"]["all_reduce"]
        assert all("xgmi_ms" in ar[c] for c in ("s", "m", "l"))     # xGMI was built and timed
        assert "xgmi1_ms" in ar["s"] and "xgmi1_ms" in ar["m"]      # one-shot for small / medium
        if tp == 2 and world > 2:
            assert "relay_ms" in ar["s"]
