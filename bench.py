#!/usr/bin/env python
"""Headline benchmark: tokens/sec (whole node) training GPT-2-small-class TP on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched with
``torch.distributed.run --nproc-per-node N`` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from env).
W untimed warmup steps, then EXACTLY K timed steps bracketed by barrier + synchronize on both
sides, elapsed = MAX over ranks, rank 0 prints ONE JSON line.

Config (BASELINE.json metric "tokens/sec (whole node), GPT-2-small TP at 1/2/4/8 MI355X"):
GPT-2 small shape in the reference block (d=768, 12 layers, 12 heads, SwiGLU ffn 2048,
vocab 50257 padded to 50304, untied head; 123.6M matmul params), seq_len 1024, bf16 compute
with fp32 master weights + Adam, random init, synthetic uniform token data.  Layout: TP
degree ``--tp`` (default ``auto`` = the model's BASELINE.json TP degree: 2 for GPT-2 small,
capped at N) with data parallelism over the remaining GPUs (``tp2dp4`` at N = 8); ``--tp N``
gives pure TP (12 heads over 8 ranks: 2 heads on ranks 0-3, 1 on ranks 4-7).  Weak scaling:
the global batch is ``--batch-per-gpu x N`` sequences (every rank does the same FLOPs per
step for every N and layout).

``--impl reference`` times the reference's eager formulation (nn.Linear/autocast, materialised
causal softmax, full-logit CE, torch.optim.Adam; tests/vanilla_model.py) on one GPU — the
in-house "reference code on MI355X" baseline recorded in BASELINE.md.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Per-GPU throughput of the reference formulation on MI355X at TP=1 (bench.py --impl reference,
# gpt2-small, seq 1024, batch 32, measured on MI355X: 183.7 ms/step); see BASELINE.md.
REFERENCE_TOKENS_PER_S_TP1 = 178376.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--batch-per-gpu", type=int, default=32)
    ap.add_argument("--global-batch", type=int, default=None, help="override (strong scaling)")
    ap.add_argument("--sp", choices=["auto", "on", "off"], default="auto",
                    help="Megatron sequence parallelism; auto = time both during the warmup steps "
                         "(TP > 1, warmup >= 4) and keep the faster, else on for TP >= 4")
    ap.add_argument("--tp", default="auto",
                    help="tensor-parallel degree (DP over the rest of the GPUs); auto = the BASELINE.json "
                         "config's TP degree for the model (gpt2-small 2, gpt2-large 4, 7B/13B 8), capped at N")
    ap.add_argument("--impl", choices=["ours", "reference"], default="ours")
    ap.add_argument("--layers", type=int, default=None, help="debug only: not a valid headline number")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--recompute", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                    help="activation recompute (layer inputs only); auto = the HBM planner's choice "
                         "(utils/memory.py: on only when the layout does not fit without it)")
    ap.add_argument("--no-pure-tp", dest="pure_tp", action="store_false",
                    help="at N > 1 with a TP x DP headline layout, skip the extra pure-TP (tp = N) measurement")
    ap.add_argument("--pure-tp-budget-s", type=float, default=float(os.environ.get("DPFS_PURE_TP_BUDGET_S", "180")),
                    help="wall-clock budget of the extra pure-TP measurement; past it every rank prints / "
                         "exits with the headline and tp_pure = {error: timeout}")
    ap.add_argument("--pg-timeout-s", type=float, default=240.0,
                    help="process-group (RCCL watchdog) timeout, well under the driver's lease")
    ap.add_argument("--graph", choices=["on", "off"], default=os.environ.get("DPFS_GRAPH", "off"),
                    help="one rank: replay the forward + backward from a HIP graph captured after the "
                         "warmup (engine.GraphTrainStep; the same kernels, launched by the graph)")
    ap.add_argument("--fp32", action="store_true",
                    help="fp32 compute (the reference's default without --bf16): the fp32-input MFMA kernel set "
                         "(ops/fp32_native.py); with --impl reference, eager fp32 without autocast. NOT the headline")
    ap.add_argument("--fp8", action="store_true",
                    help="fp8 (e4m3 / e5m2) forward and data-gradient GEMMs on hipBLASLt fp8 kernels (ops/fp8.py); "
                         "NOT the bf16 headline")
    return ap.parse_args()


# TP degree of each model's BASELINE.json config (GPT-2 small TP=2, GPT-2 large TP=4, 7B / 13B
# TP=8).  GPT-2 small at d=768 is xGMI-link-bound beyond TP 2 under weak scaling (README
# "Known limits"), so `auto` scales it out by data parallelism over TP=2 groups.
BASELINE_TP = {"gpt2-small": 2, "gpt2-large": 4, "llama2-7b": 8, "llama-13b": 8}


def resolve_tp(tp: str, model: str, world: int) -> int:
    t = BASELINE_TP.get(model, world) if tp == "auto" else int(tp)
    t = max(1, min(t, world))
    while world % t:
        t -= 1
    return t


def measure(a, tp: int, world: int, dev, first: bool):
    """Build the model on a (dp = world / tp) x tp grid, run the warmup (with the engine trial
    at TP > 1) and EXACTLY ``a.steps`` timed steps bracketed by barrier + synchronize on both
    sides.  Returns the layout's numbers (elapsed = max over ranks)."""
    from distributed_pytorch_from_scratch_amd.models import get_preset, Transformer
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    from distributed_pytorch_from_scratch_amd.engine import TrainStep
    from distributed_pytorch_from_scratch_amd.utils.dist import init_dist_env, set_seed
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm, tp_comm

    t_build = time.perf_counter()
    p = init_dist_env(rank=None, tp_size=tp, dp_size=world // tp, timeout_s=a.pg_timeout_s) if first \
        else pm.init_pgm(tp, world // tp)
    # test hooks: "raise:<rank>" | "hang:<rank>" in the pure-TP layout, "raise_head" in the
    # headline layout on every rank
    inject = os.environ.get("DPFS_BENCH_INJECT", "")
    if first and inject == "raise_head" and tp > 1:
        raise RuntimeError("injected failure in the headline layout")
    if not first and inject and inject != "raise_head" and int(inject.split(":")[1]) == dist.get_rank():
        if inject.startswith("raise"):
            raise RuntimeError("injected failure in the pure-TP layout")
        time.sleep(3600)
    tp_comm.set_fixed_shapes(True)   # synthetic fixed-shape batches on every rank

    # SP is a property of the step, not of the weights: build with the SP attributes and
    # switch the engine per step (TrainStep.sp / args.sequence_parallel).
    overrides = dict(sequence_parallel=tp > 1 and a.sp != "off")
    if a.layers:
        overrides["num_layers"] = a.layers
    if a.fp8:
        overrides["fp8"] = True
    args = get_preset(a.model, **overrides)
    T = a.seq_len
    assert T <= args.maxlen
    gb = a.global_batch or a.batch_per_gpu * world
    assert gb % p.dp_size == 0, f"global batch {gb} not divisible by DP {p.dp_size}"
    lb = gb // p.dp_size          # sequences per TP group (= per DP replica) per step
    V = args.vocab_size
    # HBM plan (utils/memory.py) before anything is allocated: recompute on only where the
    # layout does not fit without it; a layout that does not fit at all is refused here.
    from distributed_pytorch_from_scratch_amd.utils import memory as MEM
    lay = MEM.Layout(tp=tp, dp=p.dp_size, sp=bool(args.sequence_parallel), seq=T, batch=lb,
                     chunks=2 if tp > 1 else 1, compute="fp32" if a.fp32 else "bf16")
    want = {"auto": None, "on": True, "off": False}[a.recompute]
    free = MEM.device_free_bytes() if dev.type == "cuda" else None
    rc, est = MEM.plan(args, lay, free, want) if a.impl == "ours" else (False, MEM.estimate(args, lay))
    args.recompute = bool(rc)
    if dev.type == "cuda":
        torch.cuda.reset_peak_memory_stats(dev)

    set_seed(a.seed)
    # same synthetic data on every rank of a TP group, a different stream per DP replica
    g = torch.Generator(device=dev).manual_seed(1234 + 7919 * p.dp_rank)
    n_pool = 4
    # (ids, targets) as separate contiguous tensors, as a data loader hands them over
    pool = [torch.randint(0, V, (lb, T + 1), device=dev, generator=g) for _ in range(n_pool)]
    pool = [(b[:, :-1].contiguous(), b[:, 1:].contiguous()) for b in pool]
    pos = torch.arange(T, device=dev).unsqueeze(0).expand(lb, T).contiguous()

    if a.impl == "ours":
        model = Transformer.from_args(args).to(dev)
        model.reset_parameters()
        if a.fp32:
            model.set_compute_dtype(torch.float32)
        opt = FusedAdam(model.parameters(), lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.0)
        step = TrainStep(model, opt)

        def run(i):
            ids, tgt = pool[i % n_pool]
            return step(ids, pos, tgt)
    else:
        assert world == 1, "--impl reference is the single-GPU eager baseline"
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from vanilla_model import VanillaTransformer
        import torch.nn.functional as F
        model = VanillaTransformer(args.attn_dim, args.ffn_dim, args.num_heads, args.num_layers, V,
                                   args.maxlen, args.rope_theta).to(dev)
        model.cos, model.sin = model.cos.to(dev), model.sin.to(dev)
        model.reset_parameters()
        opt = torch.optim.Adam(model.parameters(), lr=3e-4)

        def run(i):
            ids, tgt = pool[i % n_pool]
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=not a.fp32):
                logits = model(ids, pos)
                loss = F.cross_entropy(logits.float().view(-1, V), tgt.reshape(-1), ignore_index=-1)
            opt.zero_grad()
            loss.backward()
            opt.step()
            return loss.detach()

    def set_cfg(cfg):
        if a.impl == "ours":
            on, chunks = cfg
            model.args.sequence_parallel = on
            step.sp = on
            model.chunks = chunks

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    # Engine configurations (SP on/off, ping-pong chunks), most likely first.  At TP > 1 the
    # warmup steps double as a trial of as many as fit (2 steps each, the first untimed:
    # first-call GEMM selection / transport choice); every rank takes the config with the
    # lowest max-over-ranks step time.  Without a trial: SP at any TP > 1 and 2 chunks (the
    # compute-only per-rank step on one MI355X, tools/tp_sim.py: TP 2 / 4 / 8 = 50.0 / 55.1 /
    # 73.8 ms without SP, 45.8 / 47.9 / 59.9 ms with it; 4 chunks cost 5-9 ms more).
    default = (tp > 1 and a.sp != "off", 2 if tp > 1 else 1)
    cands = [default]
    if a.sp == "auto":
        cands += [(default[0], 1), (not default[0], 2), (not default[0], 1), (True, 4), (False, 4)]
    else:
        cands += [(a.sp == "on", 4), (a.sp == "on", 1)]
    cands = list(dict.fromkeys(cands))
    ntrial = min(len(cands), a.warmup // 2) if a.impl == "ours" and tp > 1 else 0
    trial = {}
    i = 0
    for cfg in cands[:ntrial] if ntrial >= 2 else []:
        set_cfg(cfg)
        loss = run(i)
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        loss = run(i + 1)
        sync()
        dt_ = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(dt_, op=dist.ReduceOp.MAX)
        trial[cfg] = float(dt_.item())
        i += 2
    set_cfg(min(trial, key=trial.get) if trial else default)
    if dist.get_rank() == 0:
        print(f"[bench] tp{tp}dp{world // tp}: model built, trial {trial or '-'} "
              f"({time.perf_counter() - t_build:.1f} s)", file=sys.stderr, flush=True)
    for _ in range(a.warmup - i):
        loss = run(i)
        i += 1
    graphed = False
    if a.impl == "ours" and world == 1 and dev.type == "cuda" and a.graph == "on":
        # forward + backward replayed from one HIP graph (engine.GraphTrainStep); captured here,
        # in one more untimed warmup step
        from distributed_pytorch_from_scratch_amd.engine import GraphTrainStep
        gstep = GraphTrainStep(step)

        def run(i):
            ids, tgt = pool[i % n_pool]
            return gstep(ids, pos, tgt)
        loss = run(i)
        graphed = True
    sp_used = bool(a.impl == "ours" and model.args.sequence_parallel)
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = run(a.warmup + i)
    sync()
    dist.barrier()
    sync()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    if dist.get_rank() == 0:
        print(f"[bench] tp{tp}dp{world // tp}: {a.steps} steps in {elapsed:.2f} s "
              f"({time.perf_counter() - t_build:.1f} s since the build)", file=sys.stderr, flush=True)
    res = dict(
        value=gb * T * a.steps / elapsed, elapsed=elapsed, gb=gb, T=T, args=args,
        parallelism=f"tp{tp}" + (f"dp{p.dp_size}" if p.dp_size > 1 else "") + ("+sp" if sp_used else ""),
        final_loss=float(loss.float().item()), tp_comm=tp_comm.info(),
        chunks=model.overlap_chunks() if a.impl == "ours" else None, recompute=bool(rc),
        # the measured peak is the max over every engine configuration the trial ran: estimate
        # each of them with its own SP / chunk setting and report the max alike
        peak_mem_gb_est=round(max(MEM.estimate(args, MEM.Layout(**{**lay.__dict__, "sp": bool(k[0]),
                                                                      "chunks": int(k[1]), "recompute": bool(rc)})).gb()
                                  for k in (trial or [None])) if trial else est.gb(), 2),
        peak_mem_gb=round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2) if dev.type == "cuda" else None,
        trial={f"{'sp' if k[0] else 'nosp'}/c{k[1]}": round(1000 * v, 2) for k, v in trial.items()} or None,
        graph=graphed)
    del model, opt, pool
    if a.impl == "ours":
        del step
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    return res


def main():
    a = parse()
    if os.environ.get("DPFS_STACK_DUMP_S"):   # hang diagnosis: every rank prints its Python stacks
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["DPFS_STACK_DUMP_S"]), repeat=True)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and a.gpus > 1:
        raise SystemExit("for --gpus > 1 launch with torch.distributed.run --nproc-per-node N")
    assert world == a.gpus, f"WORLD_SIZE={world} but --gpus {a.gpus}"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    tp = resolve_tp(a.tp, a.model, world)
    if torch.cuda.is_available():
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        # DPFS_BACKEND=gloo: the multi-rank rehearsal with several ranks on one GPU
        torch.cuda.set_device(lr % torch.cuda.device_count() if os.environ.get("DPFS_BACKEND") == "gloo" else lr)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    failed = False
    try:
        head = measure(a, tp, world, dev, first=True)
    except Exception as e:   # noqa: BLE001
        # The TP x DP layout failed on every rank alike (an exception, not a hang: a hang ends
        # at the process-group timeout).  Pure data parallelism is measured for the record, but
        # it is NOT the requested layout: the line carries value = null, the DP numbers under
        # "fallback", the failure under "headline_error", and every rank exits 1.
        if world == 1 or tp == 1 or a.impl != "ours" or not dist.is_initialized():
            raise
        err = f"{type(e).__name__}: {e}"[:500]
        print(f"[bench] headline layout tp{tp}dp{world // tp} failed ({err}); measuring dp{world}",
              file=sys.stderr, flush=True)
        from distributed_pytorch_from_scratch_amd.parallel import tp_comm
        tp_comm.reset()
        head = measure(a, 1, world, dev, first=False)
        head["headline_error"] = {"parallelism": f"tp{tp}dp{world // tp}", "error": err}
        a.pure_tp = False
        failed = True
    rank = dist.get_rank()
    out = report(a, head, [head], world, dev)
    if failed:
        out["fallback"] = {"parallelism": out["config"]["parallelism"], "value": out["value"],
                           "ms_per_step": out["ms_per_step"]}
        out.update(value=None, ms_per_step=None, vs_baseline=None, tflops_per_gpu=None)
        out["mfu_vs_2.5pf_dense_bf16"] = None
        out["config"]["parallelism"] = head["headline_error"]["parallelism"]
    # The reference trains with tp_size == world_size (process_manager.py:13-15, recipe.sh TP 1 /
    # 2 / 4): at N > 1 the pure-TP layout is measured as well and reported next to the headline
    # layout (same contract: W warmup + K timed steps, max over ranks), each with its label.
    # That layout must never cost the headline: it runs after the headline's numbers are final,
    # any exception becomes tp_pure = {"error": ...}, and a per-rank timer bounds it (a hung
    # collective: rank 0 prints the headline line with tp_pure = {"error": "timeout"} and every
    # rank exits 0 before the process-group watchdog or the driver's lease fires).
    if world > 1 and tp != world and a.pure_tp:
        import threading
        lock = threading.Lock()
        done = []

        def emit(o):
            with lock:
                if not done:
                    done.append(1)
                    if rank == 0:
                        print_line(json.dumps(o))

        def expire():
            o = dict(out)
            o["tp_pure"] = {"parallelism": f"tp{world}", "error": f"timeout after {a.pure_tp_budget_s:.0f}s"}
            emit(o)
            sys.stdout.flush()
            os._exit(0)

        timer = threading.Timer(a.pure_tp_budget_s, expire)
        timer.daemon = True
        timer.start()
        err = None
        try:
            from distributed_pytorch_from_scratch_amd.parallel import tp_comm
            tp_comm.reset()            # the headline layout's xGMI buffers / communicators
            pure = measure(a, world, world, dev, first=False)
            out = report(a, head, [head, pure], world, dev)
        except Exception as e:         # noqa: BLE001 - reported, never fatal for the headline
            err = f"{type(e).__name__}: {e}"[:500]
            out = dict(out)
            out["tp_pure"] = {"parallelism": f"tp{world}", "error": err}
        timer.cancel()
        emit(out)
        # No teardown collective after the extra layout: a rank that failed alone has left its
        # peers inside a collective (their timers end them), and every rank that got here is
        # past its last collective.
        if rank == 0:
            show_gemm_choices()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    elif rank == 0:
        print_line(json.dumps(out))
    if rank == 0:
        show_gemm_choices()
    dist.barrier()
    dist.destroy_process_group()
    if failed:
        sys.exit(1)


def print_line(text: str):
    """One write(2) of the whole line: other ranks' (and libraries') output to the same pipe
    cannot land inside the driver's JSON line."""
    sys.stdout.flush()
    os.write(sys.stdout.fileno(), (text + "\n").encode())


def show_gemm_choices():
    if os.environ.get("DPFS_SHOW_GEMM") == "1":     # per-shape ours/hipBLASLt choices (ms)
        from distributed_pytorch_from_scratch_amd.ops import gemm_select
        for key, v in sorted(gemm_select.choices(with_times=True).items(), key=str):
            print(f"[gemm] {key} -> {v}", file=sys.stderr, flush=True)


def report(a, head, layouts, world, dev):
    """The driver's JSON line (headline = ``head``; ``layouts`` adds the labelled extras)."""
    args, T, gb = head["args"], head["T"], head["gb"]
    value, elapsed = head["value"], head["elapsed"]
    # The reference-formulation baseline was measured on GPT-2 small only; other shapes get null.
    base = REFERENCE_TOKENS_PER_S_TP1 if (a.model == "gpt2-small" and not a.layers) else None
    vs = None
    if base:
        # Reference measured at TP=1; for N>1 compare against ideal linear scaling of it.
        vs = value / (base * world)
    mflops = args.flops_per_token(T)
    out = {
        "metric": "tokens/sec (whole node), GPT-2-small TP at 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000 * elapsed / a.steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if a.global_batch else "weak",
        "vs_baseline": round(vs, 4) if vs else None,
        "dtype": ("fp32" if a.fp32 else "fp8-e4m3/e5m2 GEMMs + bf16" if a.fp8 else "bf16") if dev.type == "cuda"
                 else "fp32",
        "data": "synthetic (uniform random token ids), random-init weights",
        "config": {
            "model": a.model + (f"(L={a.layers})" if a.layers else ""),
            "global_batch": gb,
            "seq_len": T,
            "parallelism": head["parallelism"],
            "impl": a.impl,
            "recompute": head["recompute"],
            "fp8": bool(a.fp8),
            "params_matmul": args.matmul_params(),
            "tp_comm": head["tp_comm"],
            "chunks": head["chunks"],
            "engine_trial_ms": head["trial"],
            "hip_graph": head["graph"],
        },
        "tflops_per_gpu": round(value * mflops / world / 1e12, 2),
        "mfu_vs_2.5pf_dense_bf16": round(value * mflops / world / 2.5e15, 4),
        "final_loss": round(head["final_loss"], 4),
        "peak_mem_gb_est": head["peak_mem_gb_est"],
        "peak_mem_gb": head["peak_mem_gb"],
    }
    if head.get("headline_error"):
        out["headline_error"] = head["headline_error"]
    if world > 1:
        out["layouts"] = [{"parallelism": L["parallelism"], "value": round(L["value"], 1),
                           "ms_per_step": round(1000 * L["elapsed"] / a.steps, 3),
                           "vs_baseline": round(L["value"] / (base * world), 4) if base else None,
                           "tp_comm": L["tp_comm"], "chunks": L["chunks"], "engine_trial_ms": L["trial"]}
                          for L in layouts]
        pure = [L for L in out["layouts"] if L["parallelism"].split("+")[0] == f"tp{world}"]
        out["tp_pure"] = pure[0] if pure else None
    return out


if __name__ == "__main__":
    main()
