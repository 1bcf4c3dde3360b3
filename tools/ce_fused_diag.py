"""Diagnose ce_fused_k against the oracle: per case, the worst rows / columns and error pattern."""
import torch
from distributed_pytorch_from_scratch_amd.ops import _ext
from distributed_pytorch_from_scratch_amd.ops import reference as R

C = _ext.require()
for (M, V, valid) in [(3, 8, 5), (600, 2048, 100), (300, 1000, 997), (777, 32000, 32000), (4096, 50304, 50257)]:
    torch.manual_seed(17)
    logits = (3 * torch.randn(M, V, device="cuda")).bfloat16()
    tgt = torch.randint(0, valid, (M,), device="cuda")
    tgt[::7] = -1
    gs = (tgt >= 0).float() / max(1, int((tgt >= 0).sum()))
    ref = logits.float()
    x = logits.clone()
    st = C.ce_fused(x, tgt, gs, 0, valid, None)
    R.ce_fused(ref, tgt, gs, 0, valid, None)
    err = (x.float() - ref).abs()
    rel = (err.norm() / ref.norm()).item()
    rowerr = err.max(1).values
    bad = (rowerr > 1e-2 * ref.abs().max(1).values.clamp_min(1e-30)).nonzero().flatten()
    print(f"M={M} V={V} valid={valid}: rel {rel:.3e}; bad rows {bad.numel()} first {bad[:10].tolist()}")
    if bad.numel():
        r = bad[0].item()
        e = err[r]
        cols = (e > 1e-2 * ref[r].abs().max()).nonzero().flatten()
        print("   row", r, "bad cols", cols.numel(), cols[:16].tolist(), "got", x[r, cols[:4]].tolist(), "want", ref[r, cols[:4]].tolist(), "tgt", tgt[r].item())
