"""Time the in-place RoPE pass on the GPT-2-small QKV shape (and a LLaMA-7B one) against the
HBM floor (read + write the rotated q / k columns once).

    python tools/rope_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext, reference as R  # noqa: E402


def main():
    C = _ext.require()
    for name, M, H, hd in (("gpt2-small qkv", 32768, 12, 64), ("llama2-7b qkv", 8192, 32, 128)):
        qkv = torch.randn(M, 3 * H * hd, device="cuda").bfloat16()
        pos = torch.arange(M, device="cuda") % 1024
        tab = R.rope_table(4096, hd, 10000.0).to("cuda")
        for _ in range(3):
            C.rope_(qkv, pos, tab, 2 * H, hd, False)
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            C.rope_(qkv, pos, tab, 2 * H, hd, False)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / n
        gb = 2 * M * 2 * H * hd * 2 / 1e9
        print(f"{name}: M={M} heads={2 * H} hd={hd}: {ms * 1e3:.1f} us, {gb / ms:.2f} TB/s effective", flush=True)


if __name__ == "__main__":
    main()
