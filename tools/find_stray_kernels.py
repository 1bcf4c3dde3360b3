"""Where the non-``dpfs::`` kernels of a training step come from: torch.profiler over a few
steps of the headline bench model (GPT-2 small, TP 1; ``--fp32`` for the fp32 step), printing
every GPU kernel / memset / memcpy that is not one of ours with the Python stack of the op that
launched it.

    python tools/find_stray_kernels.py [--fp32] [--layers 2] [--steps 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from torch.profiler import profile, ProfilerActivity
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29591")
    from distributed_pytorch_from_scratch_amd.utils.dist import init_dist_env
    from distributed_pytorch_from_scratch_amd.models import get_preset, Transformer
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    from distributed_pytorch_from_scratch_amd.engine import TrainStep
    init_dist_env(rank=0, tp_size=1, world_size=1, backend="nccl")
    args = get_preset("gpt2-small", num_layers=a.layers)
    dev = torch.device("cuda", 0)
    m = Transformer.from_args(args).to(dev)
    m.reset_parameters()
    if a.fp32:
        m.set_compute_dtype(torch.float32)
    opt = FusedAdam(m.parameters(), lr=3e-4, betas=(0.9, 0.95))
    step = TrainStep(m, opt)
    T = 1024
    g = torch.Generator(device=dev).manual_seed(0)
    pool = [torch.randint(0, args.vocab_size, (a.batch, T + 1), device=dev, generator=g) for _ in range(4)]
    pool = [(b[:, :-1].contiguous(), b[:, 1:].contiguous()) for b in pool]
    pos = torch.arange(T, device=dev).unsqueeze(0).expand(a.batch, T).contiguous()
    for i in range(4):
        step(pool[i % 4][0], pos, pool[i % 4][1])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for i in range(a.steps):
            step(pool[i % 4][0], pos, pool[i % 4][1])
        torch.cuda.synchronize()
    print(f"CPU ops that launched GPU work over {a.steps} steps ({'fp32' if a.fp32 else 'bf16'}), our bindings excluded:")
    for ev in prof.key_averages():
        dt = getattr(ev, "self_device_time_total", None)
        if dt is None:
            dt = getattr(ev, "self_cuda_time_total", 0)
        if not ev.key.startswith("aten::") or dt <= 0:
            continue
        print(f"  {ev.count / a.steps:5.2f}/step  {ev.key}  ({dt / a.steps:.1f} us/step on the GPU)")
    # call sites: the Python frames (ours) of every such op that has device work of its own
    sites = {}
    for e in prof.events():
        if e.device_type.name != "CPU" or not e.name.startswith("aten::"):
            continue
        kids = [k for k in e.kernels] if hasattr(e, "kernels") else []
        if not kids:
            continue
        st = tuple(s for s in (e.stack or []) if "distributed_pytorch_from_scratch_amd" in s or "tools/" in s)[:4]
        key = (e.name, st, tuple(sorted(set(k.name[:60] for k in kids))))
        sites[key] = sites.get(key, 0) + 1
    print("call sites (op, our frames, kernels launched):")
    for (name, st, ks), n in sorted(sites.items(), key=lambda kv: -kv[1]):
        print(f"  {n / a.steps:5.2f}/step  {name}  kernels {list(ks)}")
        for s in st:
            print(f"      at {s}")


if __name__ == "__main__":
    main()
