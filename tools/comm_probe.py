"""TP collective probe: xGMI peer-memory kernels vs RCCL, per message size.

8-GPU node:  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/comm_probe.py
One GPU:     python tools/comm_probe.py --local 2      (N ranks share the device, gloo bootstrap;
             the "peer" reads are local HBM reads, so this prices the kernel, not the links)

Prints one line per (op, size, transport/blocks): ms per call and the algorithm bandwidth
(bytes of the full tensor / time) and bus bandwidth (x 2(W-1)/W for all-reduce, (W-1)/W for
reduce-scatter / all-gather, the usual nccl-tests convention).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _ms(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0) / reps


def run(rank, world, sizes_mb, reps, blocks_list):
    import torch
    import torch.distributed as dist
    from distributed_pytorch_from_scratch_amd.parallel import process_manager as pm
    from distributed_pytorch_from_scratch_amd.parallel.xgmi import XgmiComm
    g = pm.pgm.tp_group
    comm = XgmiComm(g, cap_bytes=max(sizes_mb) << 20)
    nccl = dist.get_backend(g) == "nccl"
    rows = []
    for mb in sizes_mb:
        n = (mb << 20) // 2
        n -= n % (8 * world)
        x = torch.randn(n, device="cuda").bfloat16()
        part = torch.empty(n // world, device="cuda", dtype=torch.bfloat16)
        for op, factor in (("all_reduce", 2 * (world - 1) / world), ("reduce_scatter", (world - 1) / world),
                           ("all_gather", (world - 1) / world)):
            cands = []
            for nb in blocks_list:
                def f(nb=nb):
                    comm.set_blocks(nb)
                    if op == "all_reduce":
                        comm.all_reduce(x, async_op=False)
                    elif op == "reduce_scatter":
                        comm.reduce_scatter(part, x, async_op=False)
                    else:
                        comm.all_gather(x, part, async_op=False)
                cands.append((f"xgmi/{nb}", f))
            st = comm.staging(0, (n,), torch.bfloat16) if op != "all_gather" else None
            if st is not None:          # producer wrote into a staging slot: no copy-in
                st.copy_(x)

                def fs(nb=blocks_list[-1]):
                    comm.set_blocks(nb)
                    if op == "all_reduce":
                        comm.all_reduce(st, async_op=False)
                    else:
                        comm.reduce_scatter(part, st, async_op=False)
                cands.append((f"staged/{blocks_list[-1]}", fs))
            if nccl:
                def r():
                    if op == "all_reduce":
                        dist.all_reduce(x, group=g)
                    elif op == "reduce_scatter":
                        dist.reduce_scatter_tensor(part, x, group=g)
                    else:
                        dist.all_gather_into_tensor(x, part, group=g)
                cands.append(("rccl", r))
            for name, fn in cands:
                t = torch.tensor([_ms(fn, reps)], device="cuda")
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
                ms = t.item()
                algbw = n * 2 / ms / 1e6
                rows.append(f"{op:15s} {mb:6d} MB  {name:10s} {ms:8.3f} ms  algbw {algbw:7.1f} GB/s  "
                            f"busbw {algbw * factor:7.1f} GB/s")
    comm.check()
    return rows


def _local_worker(rank, world, port, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    torch.cuda.set_device(0)
    from distributed_pytorch_from_scratch_amd.utils.dist import init_dist_env
    init_dist_env(rank=rank, tp_size=world, world_size=world, backend="gloo")
    rows = run(rank, world, args.sizes, args.reps, args.blocks)
    if rank == 0:
        print("\n".join(rows), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--local", type=int, default=0, help="N ranks on one GPU (gloo bootstrap)")
    ap.add_argument("--sizes", type=int, nargs="+", default=[8, 50, 100, 200])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--blocks", type=int, nargs="+", default=[8, 16, 32, 64])
    a = ap.parse_args()
    if a.local:
        import torch.multiprocessing as mp
        from distributed_pytorch_from_scratch_amd.utils.dist import free_port
        mp.start_processes(_local_worker, args=(a.local, free_port(), a), nprocs=a.local, start_method="spawn")
        return
    from distributed_pytorch_from_scratch_amd.utils.dist import init_dist_env
    init_dist_env(rank=None)
    import torch.distributed as dist
    rows = run(dist.get_rank(), dist.get_world_size(), a.sizes, a.reps, a.blocks)
    if dist.get_rank() == 0:
        print("\n".join(rows), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
