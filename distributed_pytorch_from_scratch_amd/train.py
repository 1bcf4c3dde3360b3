"""Training entrypoint (tensor parallel, optional DP / SP).

Reference parity: ``train.py:25-151`` — same CLI flags (``--tp_size --master_addr
--master_port --lr --warmup_steps --max_steps --log_interval --save_interval --save_dir
--reserv_last_n_ckpts --batch_size/-b --bf16 --data_path/-d --random_seed
--use_vallina_impl``), same launch model (``mp.spawn`` one process per GPU when not started by
torchrun), Adam + OneCycleLR schedule, per-rank checkpoints ``tprank-{r}_iter-{n}_loss-{x}.pth``
with keep-last-N rotation, TensorBoard scalars ``train/ce_loss`` (cumulative mean, as the
reference), ``train/lr`` and ``used_gpu_memory/tprank-{r}`` under ``{save_dir}/tprank-{r}/``.

Extensions: ``--model`` presets (reference / gpt2-small / gpt2-large / llama2-7b / llama-13b),
``--seq_len``, ``--synthetic`` data, ``--dp_size``, ``--sp`` (sequence parallel),
``--max_grad_norm``, ``--resume`` (optimizer/scheduler/RNG sidecar), throughput + MFU
logging, a per-rank heartbeat and ``--fault_inject_step`` for failure-path testing.
The loss stays on the device between log intervals (the reference syncs every step).
"""
from __future__ import annotations

import math
import os
import sys
import time
from argparse import ArgumentParser, Namespace
from dataclasses import replace

import torch
import torch.distributed as dist

from .constants import IGNORE_INDEX
from .data.dataset import get_dataloader, get_synthetic_dataloader, resume_position, seek
from .engine import TrainStep
from .models import Transformer, get_preset
from .ops.dispatch import native_fp32 as K_native_fp32
from .ops.optim import FusedAdam
from .parallel import process_manager as pm
from .utils import checkpoint as ck
from .utils import memory as MEM
from .utils.dist import destroy_dist_env, init_dist_env, set_seed, free_port
from .utils.fault import Heartbeat, maybe_inject_fault
from .utils.tb import SummaryWriter


# Dense (no sparsity) bf16 MFMA peak of one MI355X, FLOP/s.
MI355X_BF16_PEAK = 2.5e15


def _backend(use_cuda: bool) -> str:
    """RCCL on GPUs; ``DPFS_BACKEND=gloo`` runs several ranks on one GPU (the TP collectives
    then go through ``DPFS_TP_COMM``'s transports, e.g. the xGMI kernels)."""
    return os.environ.get("DPFS_BACKEND") or ("nccl" if use_cuda else "gloo")


def get_train_args(argv=None) -> Namespace:
    p = ArgumentParser()
    g = p.add_argument_group("distributed")
    g.add_argument("--tp_size", type=int, default=2)
    g.add_argument("--dp_size", type=int, default=1)
    g.add_argument("--sp", action="store_true", help="Megatron sequence parallelism")
    g.add_argument("--recompute", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                   help="activation recompute (layer inputs only); auto = the HBM planner's choice "
                        "(utils/memory.py: on only when the layout does not fit without it)")
    g.add_argument("--master_addr", type=str, default="127.0.0.1")
    g.add_argument("--master_port", type=str, default="25555")
    g = p.add_argument_group("training")
    g.add_argument("--lr", type=float, default=3e-4)
    g.add_argument("--warmup_steps", type=int, default=2000)
    g.add_argument("--max_steps", type=int, default=20000)
    g.add_argument("--log_interval", type=int, default=100)
    g.add_argument("--save_interval", type=int, default=1000)
    g.add_argument("--save_dir", type=str, default="./checkpoints")
    g.add_argument("--reserv_last_n_ckpts", type=int, default=-1)
    g.add_argument("--batch_size", "-b", type=int, default=32)
    g.add_argument("--bf16", action="store_true",
                   help="bf16 compute on the MI355X bf16 MFMA kernels (default fp32, as the reference: on the "
                        "GPU the fp32-input MFMA kernel set)")
    g.add_argument("--fp8", action="store_true",
                   help="fp8 (e4m3 / e5m2) GEMMs for the large projections, run on hipBLASLt fp8 kernels "
                        "(ops/fp8.py; quantisation on our HIP kernels); bf16 elsewhere")
    g.add_argument("--max_grad_norm", type=float, default=None)
    g.add_argument("--resume", type=str, default=None, help="checkpoint path, or 'latest'")
    g = p.add_argument_group("model")
    g.add_argument("--model", type=str, default="reference")
    g.add_argument("--seq_len", type=int, default=None, help="synthetic sequence length (default maxlen)")
    g = p.add_argument_group("data")
    g.add_argument("--data_path", "-d", type=str, default=None)
    g.add_argument("--synthetic", action="store_true")
    g = p.add_argument_group("other")
    g.add_argument("--random_seed", type=int, default=0)
    g.add_argument("--use_vallina_impl", action="store_true", help="only changes the log tag (reference)")
    g.add_argument("--fault_inject_step", type=int, default=-1)
    g.add_argument("--heartbeat_stale_s", type=float, default=300.0,
                   help="abort the job when a rank's heartbeat is older than this (must be < the "
                        "600 s RCCL timeout so a hung rank is reported instead of waited out); 0 = off")
    g.add_argument("--device", type=str, default=None, help="cuda|cpu (default: cuda if available)")
    a = p.parse_args(argv)
    if a.data_path is None and not a.synthetic:
        p.error("--data_path is required unless --synthetic")
    return a


def train(rank, args: Namespace):
    set_seed(args.random_seed)
    world = args.tp_size * args.dp_size
    use_cuda = (args.device or ("cuda" if torch.cuda.is_available() else "cpu")) == "cuda"
    if rank is None:
        p = init_dist_env(rank=None, tp_size=args.tp_size, dp_size=args.dp_size,
                          backend=_backend(use_cuda))
    else:
        p = init_dist_env(args, rank, world_size=world, backend=_backend(use_cuda))
    grank = dist.get_rank()
    dev = torch.device("cuda", torch.cuda.current_device()) if use_cuda else torch.device("cpu")
    # the reference's flag semantics (train.py:58-63): fp32 unless --bf16.  On the GPU, fp32
    # runs the native fp32 kernel set (ops/fp32_native.py: fp32-input MFMA GEMMs and flash
    # attention); --bf16 runs the bf16 MFMA kernels.
    compute_dtype = torch.bfloat16 if args.bf16 else torch.float32
    log0 = (lambda *a_: print(*a_, flush=True)) if grank == 0 else (lambda *a_: None)
    log0(f"{'Enable' if compute_dtype == torch.bfloat16 else 'Disable'} bf16 training  [{p}]")
    if use_cuda and compute_dtype == torch.float32:
        log0("fp32 on the GPU: fp32-input MFMA kernels (exact fp32, 1/16 of the bf16 MFMA rate); "
             "pass --bf16 for the bf16 MFMA kernels")

    margs = replace(get_preset(args.model), sequence_parallel=args.sp, fp8=getattr(args, "fp8", False))
    seq_len = args.seq_len or margs.maxlen
    # HBM plan before the model exists (utils/memory.py): recompute on only where the layout
    # does not fit without it; a layout that does not fit at all is refused with the numbers.
    rc = getattr(args, "recompute", "auto")
    rc = {"auto": None, "on": True, "off": False}.get(rc, rc if isinstance(rc, bool) else None)
    fp32 = compute_dtype == torch.float32
    lay = MEM.Layout(tp=p.tp_size, dp=p.dp_size, sp=args.sp, seq=seq_len, batch=args.batch_size,
                     chunks=2 if p.tp_size > 1 else 1, compute="fp32" if fp32 else "bf16",
                     materialized_attention=fp32 and not K_native_fp32())
    rc, est = MEM.plan(margs, lay, MEM.device_free_bytes(dev) if use_cuda else None, rc)
    margs = replace(margs, recompute=bool(rc))
    log0(f"HBM plan: peak {est.gb():.2f} GiB per rank estimated ({est.phase}), recompute={'on' if rc else 'off'}")
    model = Transformer.from_args(margs).to(dev)
    model.set_compute_dtype(compute_dtype)
    if margs.fp8 and not (model.fused_supported() and use_cuda):
        # fp8 GEMMs live in the explicit-schedule engines (RMSNorm models on the GPU); say so
        # instead of logging an fp8 run that trains in bf16
        raise SystemExit(f"--fp8 needs the fused engine on the GPU (RMSNorm model, CUDA); "
                         f"model norm={margs.norm!r}, device={dev.type}")
    model.reset_parameters()
    model.train()
    nparam = model.num_parameters(global_count=True)
    log0(model)
    log0(f"Number of parameters: {nparam / 1e6:.4f} million (global)")

    if args.synthetic:
        from .parallel import tp_comm
        tp_comm.set_fixed_shapes(True)   # every rank's batches have the same shape
        loader = get_synthetic_dataloader(margs.vocab_size, seq_len, args.batch_size,
                                          seed=args.random_seed + 17 * p.dp_rank)
    else:
        loader = get_dataloader(args.data_path, args.batch_size, IGNORE_INDEX, split="train",
                                maxlen=margs.maxlen, shuffle=True, seed=args.random_seed + 17 * p.dp_rank)
        assert loader.dataset.vocab_size == margs.vocab_size, "vocab size of dataset and model should be the same"

    dist.barrier()
    replicated = [q for n_, q in model.named_parameters() if ck.shard_dim(n_) is None]
    opt = FusedAdam(model.parameters(), lr=args.lr, max_grad_norm=args.max_grad_norm,
                    norm_group=p.tp_group, replicated_params=replicated)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, args.lr, total_steps=args.max_steps,
                                                pct_start=min(0.99, args.warmup_steps / max(1, args.max_steps)))
    step_fn = TrainStep(model, opt, sched)
    writer = SummaryWriter(os.path.join(args.save_dir, f"tprank-{p.tp_rank}")) if p.dp_rank == 0 else None
    hb_stale = getattr(args, "heartbeat_stale_s", 300.0)
    hb = Heartbeat(interval_s=min(30.0, max(1.0, hb_stale / 10)), stale_s=hb_stale,
                   abort_on_stale=hb_stale > 0) if hb_stale > 0 else Heartbeat(interval_s=30.0)

    start_step = 0
    if args.resume:
        path = args.resume
        if path == "latest":
            cands = ck.list_checkpoints(args.save_dir, p.tp_rank)
            path = cands[-1] if cands else None
        if path:
            ck.load_model(model, path)
            st = ck.load_resume(path, opt, None)
            start_step = ck.parse_iter(path) if st is None else int(st["step"])
            # Re-derive the LR schedule for this run's --max_steps and fast-forward it.
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                for _ in range(min(start_step, args.max_steps - 1)):
                    sched.step()
            log0(f"resumed from {path} at step {start_step}")
    # Continue the data stream where the saved run stopped (same epoch order, next batch).
    start_epoch = seek(loader, start_step)
    # the epoch holding the last step's batch, plus one
    max_epoch = max(start_epoch, resume_position(loader, max(0, args.max_steps - 1))[0]) + 1

    tag = "vanilla" if args.use_vallina_impl else f"TP-{p.tp_rank}"
    n = start_step
    accum = torch.zeros((), device=dev, dtype=torch.float64)
    accum_host = 0.0
    t_last, n_last = time.time(), n
    flops_tok = margs.flops_per_token(seq_len)
    dist.barrier()
    done = False
    for epoch in range(start_epoch, max_epoch):
        it = iter(loader)
        with hb.hold(n):           # the loader restart at an epoch boundary is not a stall
            batch = next(it, None)
        while batch is not None:
            ids = batch["input_ids"].to(dev, non_blocking=True)
            tgt = batch["target_ids"].to(dev, non_blocking=True)
            pos = batch["position_ids"].to(dev, non_blocking=True)
            maybe_inject_fault(args.fault_inject_step, n + 1, grank)
            loss = step_fn(ids, pos, tgt)
            accum += loss.double()
            n += 1
            hb.beat(n)
            if n % args.log_interval == 0:
                accum_host += float(accum.item())
                accum.zero_()
                avg = accum_host / (n - start_step)
                lr = opt.param_groups[0]["lr"]
                now = time.time()
                tps = ids.numel() * (n - n_last) * p.dp_size / (now - t_last)
                t_last, n_last = now, n
                mem = torch.cuda.memory_reserved(dev) / 1024 ** 3 if use_cuda else 0.0
                log0(f"[{tag}] Step {n}/{args.max_steps} -> Avg Loss {avg:.4f}, Lr {lr:.8f}, "
                     f"{tps:,.0f} tok/s, {tps * flops_tok / p.world_size / 1e12:.1f} TFLOP/s/GPU")
                if writer is not None:
                    writer.add_scalar("train/ce_loss", avg, n)
                    writer.add_scalar("train/lr", lr, n)
                    writer.add_scalar(f"used_gpu_memory/tprank-{p.tp_rank}", mem, n)
                    writer.add_scalar("throughput/tokens_per_s", tps, n)
                    # model FLOPs utilisation vs the MI355X dense bf16 peak (2.5 PFLOP/s per GPU)
                    writer.add_scalar("throughput/mfu", tps * flops_tok / p.world_size / MI355X_BF16_PEAK, n)
                    for k_, v_ in step_fn.timings().items():
                        writer.add_scalar(f"time/{k_}", v_, n)
                    writer.flush()
            if n % args.save_interval == 0:
                accum_host += float(accum.item())
                accum.zero_()
                avg = accum_host / (n - start_step)
                with hb.hold(n):       # the save and the barrier behind it take no steps
                    if p.dp_rank == 0:
                        path = ck.save_checkpoint(model, args.save_dir, p.tp_rank, n, avg, opt, sched,
                                                  keep_last_n=args.reserv_last_n_ckpts)
                        print(f"[TP rank {p.tp_rank}]: Model saved to {path}", flush=True)
                    dist.barrier()
            if n >= args.max_steps:
                done = True
                break
            batch = next(it, None)
        log0(f"Epoch {epoch + 1}/{max_epoch} finished.")
        if done:
            break
    log0(f"Training finished (total steps: {n}).")
    if writer is not None:
        writer.close()
    hb.stop()
    dist.barrier()
    destroy_dist_env()


def main(argv=None):
    args = get_train_args(argv)
    if "WORLD_SIZE" in os.environ and "RANK" in os.environ:
        train(None, args)   # torchrun: one process per GPU already
        return
    import torch.multiprocessing as mp
    os.environ.setdefault("MASTER_ADDR", args.master_addr)
    mp.spawn(train, args=(args,), nprocs=args.tp_size * args.dp_size, join=True)


if __name__ == "__main__":
    main()
