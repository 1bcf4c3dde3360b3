"""Attention backward outputs of the GPT-2-small layer shape for a bitwise A/B of two builds.

    AB_LABEL=new python tools/attn_bwd_dump.py      -> gpurun_out/attn_bwd_new.pt
    python tools/attn_bwd_dump.py --compare new old  (bitwise equal?)
"""
import argparse
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "gpurun_out")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compare", nargs=2, default=None)
    ap.add_argument("--hd", type=int, default=64)
    a = ap.parse_args()
    if a.compare:
        x, y = (torch.load(os.path.join(OUT, f"attn_bwd_{n}_hd{a.hd}.pt"), weights_only=True) for n in a.compare)
        for k in x:
            print(f"hd {a.hd} {k}: bitwise equal {torch.equal(x[k], y[k])}, max|diff| "
                  f"{(x[k].float() - y[k].float()).abs().max().item():.3e}")
        return
    from distributed_pytorch_from_scratch_amd.ops import _ext
    C = _ext.require()
    torch.manual_seed(0)
    B, T, H, hd = 4, 1024, 12 * 64 // a.hd, a.hd
    qkv = torch.randn(B * T, 3 * H * hd, device="cuda").bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    scale = 1 / math.sqrt(hd)
    o, lse = C.attn_fwd(q, k, v, scale, True)
    do = torch.randn_like(o)
    d = torch.empty_like(qkv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv)
    torch.cuda.synchronize()
    os.makedirs(OUT, exist_ok=True)
    torch.save({"o": o.cpu(), "lse": lse.cpu(), "dq": dq.cpu(), "dk": dk.cpu(), "dv": dv.cpu()},
               os.path.join(OUT, f"attn_bwd_{os.environ.get('AB_LABEL', 'x')}_hd{hd}.pt"))
    print(f"saved hd {hd}")


if __name__ == "__main__":
    main()
