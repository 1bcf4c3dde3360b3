import torch
from distributed_pytorch_from_scratch_amd.models import Transformer, get_preset
from distributed_pytorch_from_scratch_amd.ops import gemm_select as GS
from distributed_pytorch_from_scratch_amd.ops import _ext
C = _ext.require()
orig = GS.gemm_tn_group
def rec(k, items):
    A = [a for a, _, _, _ in items]; B = [b for _, b, _, _ in items]; O = [o for _, _, o, _ in items]
    acc = [int(bool(x)) for *_, x in items]
    print("group", [(tuple(a.shape), a.stride(), tuple(b.shape), b.stride(), tuple(o.shape), o.stride(), o.is_contiguous(), x) for a, b, o, x in items])
    print("  direct call ->", C.gemm_tn_group(A, B, [torch.empty_like(o) for o in O], acc))
    return orig(k, items)
GS.gemm_tn_group = rec
args = get_preset("gpt2-small", num_layers=1)
m = Transformer.from_args(args).cuda()
ids = torch.randint(0, args.vocab_size, (4, 1024), device="cuda")
pos = torch.arange(1024, device="cuda").repeat(4, 1)
m.loss(ids, pos, ids, unit_grad=True).backward()
torch.cuda.synchronize()
print("ok")
