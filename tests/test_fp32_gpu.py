"""fp32 training on the GPU (the reference's default without --bf16, /root/reference/train.py:
58-63): the engines run the native fp32 kernel set on the device (ops.dispatch.K with an fp32
compute dtype -> ops/fp32_native.py: fp32-input MFMA GEMMs and flash attention), and TP stays
numerically transparent -- the SURVEY §0 invariant checked on the MI355X: TP = 1 / 2 / 4 (and
SP) losses over Adam steps equal the vanilla fp32 model's on the CPU to 2e-5.  Ranks share one
GPU over gloo."""
import pytest
import torch

from dist_helpers import run_distributed
from test_model_tp_equivalence import _batch, _train_vanilla

# head_dim 32 (the native fp32 attention's smallest), 4 heads: one per rank at TP 4
CFG = dict(attn_dim=128, ffn_dim=256, num_heads=4, num_layers=2, vocab_size=96, maxlen=64)

pytestmark = pytest.mark.gpu


def _train_gpu(rank, world, cfg, steps, sp):
    torch.cuda.set_device(0)
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    m = Transformer.from_args(ModelArgs(**cfg, vocab_pad_to=1, sequence_parallel=sp))
    set_seed(0)
    m.reset_parameters()            # on the CPU: the vanilla model's RNG order
    m = m.cuda().set_compute_dtype(torch.float32)
    from distributed_pytorch_from_scratch_amd.ops import dispatch, fp32_native
    assert dispatch.K(m.embedding.weight, torch.float32) is fp32_native   # the native fp32 kernels
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for s in range(steps):
        ids, pos, tgt = (t.cuda() for t in _batch(cfg["vocab_size"], 2, 16, seed=100 + s))
        loss = m.loss(ids, pos, tgt)
        opt.zero_grad()
        loss.backward()
        if sp:
            from distributed_pytorch_from_scratch_amd.parallel.grad_sync import allreduce_sequence_parallel_grads
            allreduce_sequence_parallel_grads(m)
        opt.step()
        losses.append(loss.item())
    return losses


@pytest.mark.parametrize("world,sp", [(1, False), (2, False), (4, False), (2, True)])
def test_fp32_gpu_tp_transparent(world, sp):
    van, _ = _train_vanilla(CFG, 3)
    res = run_distributed(_train_gpu, world, CFG, 3, sp, timeout=240)
    for r in range(world):
        assert torch.allclose(torch.tensor(res[r]), torch.tensor(van), atol=2e-5), (res[r], van)


def _train_gpu_bf16_no_lib(rank, world, cfg, steps):
    """bf16 compute with every torch GEMM entry point poisoned: an uneven vocab shard (501 / 500
    rows at TP 2) must run on our kernels (gemm_select -> the any-alignment gemm_f32 path)."""
    import torch.nn.functional as F
    torch.cuda.set_device(0)
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    m = Transformer.from_args(ModelArgs(**cfg, vocab_pad_to=1))
    set_seed(0)
    m.reset_parameters()
    m = m.cuda().set_compute_dtype(torch.bfloat16)

    def poisoned(*a, **k):
        raise AssertionError("torch GEMM reached in the bf16 step")
    saved = (F.linear, torch.mm, torch.matmul, torch.addmm)
    F.linear = torch.mm = torch.matmul = torch.addmm = poisoned
    try:
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        losses = []
        for s in range(steps):
            ids, pos, tgt = (t.cuda() for t in _batch(cfg["vocab_size"], 2, 16, seed=100 + s))
            loss = m.loss(ids, pos, tgt)
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
    finally:
        F.linear, torch.mm, torch.matmul, torch.addmm = saved
    return losses


def test_bf16_uneven_vocab_native_gemms():
    cfg = dict(attn_dim=128, ffn_dim=256, num_heads=2, num_layers=2, vocab_size=1001, maxlen=64)
    van, _ = _train_vanilla(cfg, 3)
    res = run_distributed(_train_gpu_bf16_no_lib, 2, cfg, 3, timeout=240)
    for r in range(2):
        assert all(x == x and abs(x) < 20 for x in res[r]), res[r]
        assert torch.allclose(torch.tensor(res[r]), torch.tensor(van), atol=5e-2), (res[r], van)   # bf16
