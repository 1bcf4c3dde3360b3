"""Reference-API RoPE helpers (models/model.py:17-46 parity) vs the fused kernel-form path."""
import torch

from distributed_pytorch_from_scratch_amd.models import apply_rotary_pos_emb, get_cos_sin, rotate_half
from distributed_pytorch_from_scratch_amd.models.rope import half_table_from_full
from distributed_pytorch_from_scratch_amd.ops import reference as R


def test_rotate_half():
    x = torch.arange(8.0)
    assert torch.equal(rotate_half(x), torch.tensor([-4.0, -5, -6, -7, 0, 1, 2, 3]))


def test_apply_rotary_matches_kernel_form():
    torch.manual_seed(0)
    B, H, T, hd = 2, 3, 10, 16
    cos, sin = get_cos_sin(32, hd, 10000.0, dtype=torch.float32, device="cpu")
    tab = R.rope_table(32, hd, 10000.0)
    assert torch.allclose(half_table_from_full(cos, sin), tab)
    pos = torch.randint(0, 32, (B, T))
    q, k = torch.randn(B, H, T, hd), torch.randn(B, H, T, hd)
    qe, ke = apply_rotary_pos_emb(q, k, cos[pos], sin[pos])
    # kernel form: packed rows [q heads | k heads] of shape (B*T, 2*H*hd)
    packed = torch.cat([q.transpose(1, 2).reshape(B * T, H * hd), k.transpose(1, 2).reshape(B * T, H * hd)], 1)
    R.rope_(packed, pos.reshape(-1), tab, 2 * H, hd, False)
    assert torch.allclose(packed[:, :H * hd], qe.transpose(1, 2).reshape(B * T, -1), atol=1e-5)
    assert torch.allclose(packed[:, H * hd:], ke.transpose(1, 2).reshape(B * T, -1), atol=1e-5)
    # inverse rotation undoes it
    R.rope_(packed, pos.reshape(-1), tab, 2 * H, hd, True)
    assert torch.allclose(packed[:, :H * hd], q.transpose(1, 2).reshape(B * T, -1), atol=1e-5)


def test_dtype_env_selects_cpu_activation_dtype(monkeypatch):
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    m = Transformer.from_args(ModelArgs(attn_dim=32, ffn_dim=64, num_heads=2, num_layers=1, vocab_size=64,
                                        maxlen=16, vocab_pad_to=1))
    monkeypatch.setenv("DTYPE", "bfloat16")
    assert m.act_dtype(torch.device("cpu")) == torch.bfloat16
    cos, _ = get_cos_sin(4, 8, 10000.0, device="cpu")
    assert cos.dtype == torch.bfloat16
    monkeypatch.setenv("DTYPE", "float32")
    assert m.act_dtype(torch.device("cpu")) == torch.float32
