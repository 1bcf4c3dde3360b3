"""xGMI peer-memory collectives (csrc/comm/xgmi.hip) on one MI355X with several ranks.

The ranks are processes sharing one GPU: the IPC mapping, the per-workgroup epoch barriers,
the two-shot all-reduce, reduce-scatter, all-gather, chunking past the buffer capacity and the
engine's use of them are the same code paths as across the 8 GPUs of a node (only the link
speed differs).  Bootstrap goes over gloo (RCCL refuses two ranks on one device).  Expected
values are computed in fp32 on the host from the same rank-seeded inputs.
"""
import os

import pytest
import torch

from dist_helpers import run_distributed

pytestmark = pytest.mark.gpu


def _inputs(rank, n, dtype, seed=0):
    g = torch.Generator().manual_seed(1000 * seed + rank)
    return torch.randn(n, generator=g).to(dtype)


def _collectives(rank, world, cases, cap_mb):
    torch.cuda.set_device(0)
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm
    from distributed_pytorch_from_scratch_amd.parallel.xgmi import XgmiComm
    comm = XgmiComm(pm.pgm.tp_group, cap_bytes=cap_mb << 20, timeout_s=30.0)
    out = {}
    for i, (op, n, dt) in enumerate(cases):
        dtype = getattr(torch, dt)
        x = _inputs(rank, n, dtype, seed=i).cuda()
        if op == "ar":
            y = x.clone()
            comm.all_reduce(y, async_op=True).wait()
            y2 = x.clone()                      # back-to-back calls reuse the buffers
            comm.all_reduce(y2, async_op=False)
            # one-shot (one barrier, every peer's whole message; two calls in a row alternate
            # its input regions), falling back to two-shot past its capacity: same values
            y3, y4 = x.clone(), x.clone()
            comm.all_reduce(y3, async_op=True, one_shot=True).wait()
            comm.all_reduce(y4, async_op=False, one_shot=True)
            st = comm.staging(i % comm.nslots, (n,), dtype)   # produced in a staging slot
            if st is not None:
                st.copy_(x)
                comm.all_reduce(st, async_op=False)
                st = st.cpu()
            res = (y.cpu(), y2.cpu(), y3.cpu(), y4.cpu()) + ((st,) if st is not None else ())
        elif op == "rs":
            y = torch.empty(n // world, dtype=dtype, device="cuda")
            comm.reduce_scatter(y, x, async_op=False)
            st = comm.staging(1, (n,), dtype)
            st.copy_(x)
            y2 = torch.empty_like(y)
            comm.reduce_scatter(y2, st, async_op=False)
            res = (y.cpu(), y2.cpu())
        else:
            y = torch.empty(n * world, dtype=dtype, device="cuda")
            comm.all_gather(y, x, async_op=False)
            res = (y.cpu(),)
        out[i] = res
    torch.cuda.synchronize()
    assert comm.error() == 0
    comm.close()
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_collectives_match_fp32_sums(world):
    cases = [("ar", 8 * 1000, "bfloat16"), ("ar", 4096 * 768 + 8, "bfloat16"), ("ar", 12288, "float32"),
             ("ar", 3 * (1 << 20), "bfloat16"),          # > 4 MiB capacity: chunked
             ("rs", world * 8 * 517, "bfloat16"), ("ag", 8 * 301, "bfloat16"), ("ag", 4 * 77, "float32")]
    res = run_distributed(_collectives, world, cases, 4, tp_size=world)
    for i, (op, n, dt) in enumerate(cases):
        dtype = getattr(torch, dt)
        xs = [_inputs(r, n, dtype, seed=i) for r in range(world)]
        total = torch.stack([x.float() for x in xs]).sum(0)
        for r in range(world):
            got = res[r][i]
            if op == "ar":
                for y in got:
                    assert torch.allclose(y.float(), total, atol=2e-2, rtol=1e-2), (op, n, r)
                # fp32 sum in rank order, rounded once: identical on every rank, and the one-shot
                # form bit-identical to the two-shot one
                assert torch.equal(got[0], res[0][i][0]) and all(torch.equal(got[0], y) for y in got[1:])
            elif op == "rs":
                sl = total.view(world, -1)[r]
                assert torch.allclose(got[0].float(), sl, atol=2e-2, rtol=1e-2), (op, n, r)
                assert torch.equal(got[0], got[1])   # staged input: same result, no copy-in
            else:
                assert torch.equal(got[0], torch.cat(xs)), (op, n, r)


def _engine(rank, world, heads, sp, recompute=False):
    from test_multiproc_gpu import _train
    return _train(rank, world, world, 1, heads, "cuda", sp, recompute)


@pytest.mark.parametrize("world,sp,rc", [(2, False, False), (2, True, False), (4, True, False),
                                         (2, False, True), (2, True, True)])
def test_engine_over_xgmi_follows_single_rank(monkeypatch, world, sp, rc):
    """The fused engines with their TP collectives on the xGMI kernels (all-reduce; or
    reduce-scatter / all-gather under sequence parallelism) track the single-rank trajectory
    (same check as test_multiproc_gpu); ``rc``: with activation recompute, whose rebuilt
    forward issues its own collectives between the backward's (staging-slot reuse)."""
    from test_multiproc_gpu import _ref
    heads = 12
    ref = _ref(heads)
    monkeypatch.setenv("DPFS_TP_COMM", "xgmi")
    res = run_distributed(_engine, world, heads, sp, rc, tp_size=world)
    for r, losses in res.items():
        for a, b in zip(losses, ref):
            assert abs(a - b) < 2e-2 * max(1.0, abs(b)), (r, losses, ref)
    assert len({tuple(v) for v in res.values()}) == 1


def _setup_failure(rank, world, where):
    """One rank's allocation (``create``) or peer mapping (``open``) fails: every rank must raise
    (no rank left blocked in the next collective), and tp_comm's builder drops xGMI everywhere."""
    torch.cuda.set_device(0)
    from distributed_pytorch_from_scratch_amd.ops import _ext
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm, tp_comm
    from distributed_pytorch_from_scratch_amd.parallel.xgmi import XgmiComm
    C = _ext.require()

    class Faulty:   # the native module with one entry point failing on rank 1
        def __getattr__(self, name):
            f = getattr(C, name)
            if name == f"xgmi_{where}" and rank == 1:
                def fail(*a, **k):
                    raise RuntimeError(f"injected {name} failure")
                return fail
            return f
    real = _ext.require
    _ext.require = lambda: Faulty()
    try:
        try:
            XgmiComm(pm.pgm.tp_group, cap_bytes=1 << 20, timeout_s=10.0)
            raised = False
        except RuntimeError as e:
            raised = "every rank" in str(e)
        built = tp_comm._build("xgmi", pm.pgm.tp_group, forced=False)
    finally:
        _ext.require = real
    return dict(raised=raised, built=built is not None)


@pytest.mark.parametrize("where", ["create", "open"])
def test_xgmi_setup_failure_is_group_consistent(where):
    res = run_distributed(_setup_failure, 2, where, tp_size=2, timeout=120)
    assert all(v["raised"] for v in res.values()), res
    assert not any(v["built"] for v in res.values()), res
