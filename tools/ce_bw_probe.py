"""Bandwidth bound of the one-pass CE (ce_fused_k) at the GPT-2-small head shape: ms per call of
ce_fused on [32768, 50304] bf16 logits (reads them once, writes d logits once, in place) against
a same-size device copy (torch copy_: one read + one write of the same bytes) and a read-only
reduction, same process, interleaved.  Run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE for the
bytes each kernel moves."""
import torch
from distributed_pytorch_from_scratch_amd.ops import _ext

C = _ext.require()
M, V, VALID = 32768, 50304, 50257
torch.manual_seed(0)
x = (3 * torch.randn(M, V, device="cuda")).bfloat16()
y = torch.empty_like(x)
tgt = torch.randint(0, VALID, (M,), device="cuda")
gs = torch.full((M,), 1.0 / M, device="cuda")
db = torch.empty(V, device="cuda")
nbytes = x.numel() * x.element_size()


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {"ce_fused": [], "copy": [], "sum": []}
for _ in range(3):
    res["ce_fused"].append(t(lambda: C.ce_fused(x, tgt, gs, 0, VALID, db)))
    res["copy"].append(t(lambda: y.copy_(x)))
    res["sum"].append(t(lambda: x.sum(dtype=torch.float32)))
for k, v in res.items():
    ms = min(v)
    moved = nbytes * (1 if k == "sum" else 2)
    print(f"{k:9s} {ms:.3f} ms  {moved / ms / 1e9:.2f} TB/s  ({moved / 1e9:.2f} GB moved)", flush=True)
