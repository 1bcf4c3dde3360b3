"""Training steps of a 2-layer GPT-2-small-shape model with the TN (weight-gradient) main loop's
barrier-row hook at 0 / 1 / 2: parameters after two Adam steps must be bit-identical.

    python tools/tn_br_bitwise.py [--tokens-per-seq 1024 --batch 8]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29556")
    from distributed_pytorch_from_scratch_amd.ops import _ext
    C = _ext.require()
    from distributed_pytorch_from_scratch_amd.utils.dist import init_dist_env, set_seed
    from distributed_pytorch_from_scratch_amd.models import get_preset, Transformer
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    from distributed_pytorch_from_scratch_amd.engine import TrainStep
    init_dist_env(rank=0, tp_size=1, world_size=1)
    dev = torch.device("cuda", 0)
    res = {}
    for br in (0, 1, 2):
        C.gemm4_br_tn(br)
        set_seed(0)
        args = get_preset("gpt2-small", num_layers=2)
        model = Transformer.from_args(args).to(dev)
        model.reset_parameters()
        step = TrainStep(model, FusedAdam(model.parameters(), lr=1e-3))
        g = torch.Generator(device=dev).manual_seed(1)
        ids = torch.randint(0, args.vocab_size, (a.batch, a.seq + 1), device=dev, generator=g)
        pos = torch.arange(a.seq, device=dev).unsqueeze(0).expand(a.batch, a.seq).contiguous()
        for _ in range(2):
            step(ids[:, :-1].contiguous(), pos, ids[:, 1:].contiguous())
        torch.cuda.synchronize()
        res[br] = [p.detach().clone() for p in model.parameters()]
    C.gemm4_br_tn(0)
    for br in (1, 2):
        print(f"br_tn {br}: parameters bitwise equal to br_tn 0: "
              f"{all(torch.equal(x, y) for x, y in zip(res[0], res[br]))}", flush=True)


if __name__ == "__main__":
    main()
