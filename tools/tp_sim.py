"""Per-rank compute time of a TP = N training step, measured on ONE GPU.

Builds the model exactly as TP rank ``--rank`` of an N-way group would (head / ffn / vocab
shards, per-rank batch = ``batch_per_gpu * N`` for the weak-scaling bench) and runs the fused
engine with every TP collective replaced by a no-op.  The result is the compute-only step
time of that rank: the floor a perfectly overlapped N-GPU step can reach, and how much of it
the replicated work (norms / residuals without SP) costs.  Numerics are meaningless (partial
sums are never combined); only timing is reported.

    python tools/tp_sim.py --tp 8 [--rank 0] [--steps 5]
    python tools/tp_sim.py --tp 2 --emulate-comm 64 [--comm-blocks 32]

``--emulate-comm GBPS`` replaces each no-op collective by a stand-in kernel on a high-priority
side stream: the xGMI kernels' grid (``--comm-blocks`` workgroups of 1024 threads) resident
for the collective's modelled duration at GBPS per link and direction (a W-rank two-shot
all-reduce moves 2 x bytes / W over each link, a reduce-scatter or all-gather bytes / W), and
the engine waits for it exactly as for the real collective.  The difference to the no-op floor
is what losing those CUs to a collective costs the persistent / stream-K GEMMs and the rest of
the step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class SimPGM:
    def __init__(self, tp, rank):
        self.tp_size, self.tp_rank = tp, rank
        self.dp_size, self.dp_rank = 1, 0
        self.global_rank, self.world_size = 0, 1      # world 1: init broadcasts are skipped
        self.tp_group = self.dp_group = None
        self.tp_ranks, self.dp_ranks = list(range(tp)), [0]
        self.tp_src_rank = 0
        self.backend = "gloo"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--batch-per-gpu", type=int, default=32)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--configs", default="nosp:2,sp:2,sp:4,nosp:4")
    ap.add_argument("--cprofile", action="store_true", help="host-side profile of one step per config")
    ap.add_argument("--head-start-ms", type=float, default=0.0,
                    help="queue a GPU sleep of this length before each timed step and subtract it: "
                         "with the host that far ahead, launch latency cannot starve the GPU")
    ap.add_argument("--emulate-comm", type=float, default=0.0,
                    help="GB/s per xGMI link: collectives become CU-holding stand-ins of the modelled duration")
    ap.add_argument("--comm-blocks", type=int, default=int(os.environ.get("DPFS_XGMI_BLOCKS", "32")))
    ap.add_argument("--mem-check", action="store_true",
                    help="also print the HBM planner's per-rank estimate of each layout (utils/memory.py; the "
                         "xGMI staging term excluded: the simulation allocates none) against the measured peak")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29581")
    dist.init_process_group("gloo", rank=0, world_size=1)
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm, tp_comm
    from distributed_pytorch_from_scratch_amd.models import fused_engine_sp  # noqa: F401
    pm.pgm = SimPGM(a.tp, a.rank)
    n = a.tp
    if a.emulate_comm > 0:
        from distributed_pytorch_from_scratch_amd.ops import _ext
        C = _ext.require()
        side = torch.cuda.Stream(priority=-1)
        stats = {"calls": 0, "us": 0.0}

        class _Work:
            def __init__(self, ev):
                self.ev = ev

            def wait(self):
                torch.cuda.current_stream().wait_event(self.ev)

        def _emulate(nbytes, per_link_factor):
            us = per_link_factor * nbytes / n / (a.emulate_comm * 1e3)   # bytes / (GB/s) -> us
            stats["calls"] += 1
            stats["us"] += us
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                C.occupy(a.comm_blocks, us)
                ev = torch.cuda.Event()
                ev.record(side)
            return _Work(ev)

        tp_comm.all_reduce = lambda t, async_op=True: _emulate(t.numel() * t.element_size(), 2.0)
        tp_comm.reduce_scatter = lambda out, inp, async_op=True: _emulate(inp.numel() * inp.element_size(), 1.0)
        tp_comm.all_gather = lambda out, inp, async_op=True: _emulate(out.numel() * out.element_size(), 1.0)
    else:
        stats = None
        tp_comm.all_reduce = lambda t, async_op=True: None
        tp_comm.reduce_scatter = lambda out, inp, async_op=True: None
        tp_comm.all_gather = lambda out, inp, async_op=True: None
    dist.all_gather_into_tensor = lambda out, inp, group=None, async_op=False: out.view(n, -1).copy_(
        inp.reshape(1, -1).expand(n, -1))
    dist.all_reduce = lambda t, *args, **kw: None
    from distributed_pytorch_from_scratch_amd.models import get_preset, Transformer
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    from distributed_pytorch_from_scratch_amd.engine import TrainStep
    dev = torch.device("cuda", 0)
    args = get_preset(a.model, sequence_parallel=True)
    model = Transformer.from_args(args).to(dev)
    model.reset_parameters()
    opt = FusedAdam(model.parameters(), lr=3e-4)
    step = TrainStep(model, opt)
    B, T = a.batch_per_gpu * n, a.seq_len
    ids = torch.randint(0, args.vocab_size, (B, T + 1), device=dev)
    pos = torch.arange(T, device=dev).unsqueeze(0).expand(B, T).contiguous()
    res = {}
    for cfg in a.configs.split(","):
        sp, c, *rest = cfg.split(":")       # sp:2 or sp:2:rc (activation recompute)
        model.args.sequence_parallel = step.sp = sp == "sp"
        model.args.recompute = "rc" in rest
        model.chunks = int(c)
        torch.cuda.reset_peak_memory_stats()
        for _ in range(2):
            step(ids[:, :-1], pos, ids[:, 1:])
        torch.cuda.synchronize()
        sleep_cycles, sleep_ms = 0, 0.0
        if a.head_start_ms > 0:          # calibrate torch.cuda._sleep (clock cycles -> ms)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            torch.cuda._sleep(10_000_000)
            e1.record()
            e1.synchronize()
            sleep_cycles = int(10_000_000 * a.head_start_ms / e0.elapsed_time(e1))
        ev = []
        t0 = time.perf_counter()
        for _ in range(a.steps):
            if sleep_cycles:
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(sleep_cycles)
                e0.record()
                step(ids[:, :-1], pos, ids[:, 1:])
                e1.record()
                ev.append((e0, e1))
            else:
                step(ids[:, :-1], pos, ids[:, 1:])
        torch.cuda.synchronize()
        res[cfg] = round(1000 * (time.perf_counter() - t0) / a.steps, 2)
        if ev:                           # GPU time of the step alone (sleep excluded)
            res[cfg] = round(sum(x.elapsed_time(y) for x, y in ev) / len(ev), 2)
        # host enqueue time of one step (returns before the GPU finishes unless the host blocks)
        t1 = time.perf_counter()
        if a.cprofile:
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
        step(ids[:, :-1], pos, ids[:, 1:])
        host_ms = round(1000 * (time.perf_counter() - t1), 2)
        if a.cprofile:
            pr.disable()
            pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(25)
        torch.cuda.synchronize()
        line = {"tp": n, "rank": a.rank, "config": cfg, "ms_per_step": res[cfg], "tokens": B * T,
                "host_ms": host_ms, "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)}
        if a.mem_check:
            from distributed_pytorch_from_scratch_amd.utils import memory as MEM
            est = MEM.estimate(args, MEM.Layout(tp=n, sp=sp == "sp", seq=T, batch=B, chunks=int(c),
                                                recompute="rc" in rest, tp_rank=a.rank))
            est_b = est.peak - est.parts["xgmi_staging"]
            meas = torch.cuda.max_memory_allocated()
            line.update(est_gb=round(est_b / 2**30, 2), est_over_measured=round(est_b / meas, 3))
        if stats is not None:
            calls = stats["calls"] / max(1, a.steps + 3)
            line.update(emulate_comm_gbps=a.emulate_comm, comm_blocks=a.comm_blocks,
                        comm_ms_per_step_modelled=round(stats["us"] / max(1, a.steps + 3) / 1000, 2),
                        comm_calls_per_step=round(calls, 1))
            stats["calls"], stats["us"] = 0, 0.0
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
    if os.environ.get("DPFS_SHOW_GEMM") == "1":     # per-shape GEMM choices (ms)
        from distributed_pytorch_from_scratch_amd.ops import gemm_select
        for key, v in sorted(gemm_select.choices(with_times=True).items(), key=str):
            print(f"[gemm] {key} -> {v}", file=sys.stderr, flush=True)
