"""HBM planner arithmetic (utils/memory.py) on the CPU: parameter bytes match the model, the
activation terms scale as the layout says, and the plan turns recompute on / refuses layouts
against a budget (the 13B seq-8192 preset on one 288 GB MI355X needs recompute)."""
import pytest

from distributed_pytorch_from_scratch_amd.models import get_preset
from distributed_pytorch_from_scratch_amd.utils import memory as MEM

GB288 = 288 * 10 ** 9


@pytest.mark.parametrize("name", ["plumbing", "reference", "gpt2-small", "llama2-7b", "llama-13b"])
def test_param_bytes_match_the_model_size(name):
    a = get_preset(name)
    e = MEM.estimate(a, MEM.Layout(tp=1, seq=256, batch=1))
    assert e.parts["master_fp32"] == 4 * a.num_params()
    assert e.parts["adam_m_v_fp32"] == 8 * a.num_params()
    assert e.parts["grad_arena_fp32"] == 4 * a.num_params()


def test_param_count_matches_a_built_model():
    import torch
    from distributed_pytorch_from_scratch_amd.models import Transformer
    a = get_preset("plumbing")
    m = Transformer.from_args(a)
    n = sum(p.numel() for p in m.parameters())
    w2d = sum(p.numel() for p in m.parameters() if p.dim() == 2)
    e = MEM.estimate(a, MEM.Layout(tp=1, seq=64, batch=2))
    assert e.parts["master_fp32"] == 4 * n and e.parts["shadow_bf16"] == 2 * w2d
    del torch


def test_sharding_and_sp_and_recompute_shrink_the_right_terms():
    a = get_preset("gpt2-small")
    e1 = MEM.estimate(a, MEM.Layout(tp=1, seq=1024, batch=32))
    e2 = MEM.estimate(a, MEM.Layout(tp=2, seq=1024, batch=32))
    e2sp = MEM.estimate(a, MEM.Layout(tp=2, sp=True, seq=1024, batch=32))
    e1rc = MEM.estimate(a, MEM.Layout(tp=1, seq=1024, batch=32, recompute=True))
    # weights (all sharded except norms / row biases) roughly halve at TP 2
    assert 0.49 < e2.parts["master_fp32"] / e1.parts["master_fp32"] < 0.52
    # activations: the per-head / per-ffn terms halve, the residual stream does not (no SP)
    assert e2.parts["activations"] < e1.parts["activations"]
    assert e2sp.parts["activations"] < e2.parts["activations"]
    assert e1rc.parts["activations"] < e1.parts["activations"] / 10
    # doubling the tokens doubles the activations
    e1b = MEM.estimate(a, MEM.Layout(tp=1, seq=1024, batch=64))
    assert e1b.parts["activations"] == 2 * e1.parts["activations"]


def test_plan_gpt2_small_fits_without_recompute():
    rc, e = MEM.plan(get_preset("gpt2-small"), MEM.Layout(tp=1, seq=1024, batch=32), GB288)
    assert rc is False and e.gb() < 60


def test_plan_13b_seq8192_picks_recompute_on_one_gpu():
    a = get_preset("llama-13b")
    lay = MEM.Layout(tp=1, seq=8192, batch=1)
    rc, e = MEM.plan(a, lay, GB288)
    assert rc is True
    # without recompute it does not fit: forcing it off is refused with the numbers
    with pytest.raises(MEM.DoesNotFit) as ei:
        MEM.plan(a, lay, GB288, recompute=False)
    assert "GiB" in str(ei.value) and "with recompute" in str(ei.value)
    # at TP 8 (BASELINE config 5) it fits without recompute
    rc8, _ = MEM.plan(a, MEM.Layout(tp=8, seq=8192, batch=1), GB288)
    assert rc8 is False


def test_plan_refuses_what_does_not_fit_at_all():
    with pytest.raises(MEM.DoesNotFit):
        MEM.plan(get_preset("llama-13b"), MEM.Layout(tp=1, seq=8192, batch=1), 80 * 10 ** 9)


def test_plan_without_budget_never_refuses():
    rc, e = MEM.plan(get_preset("llama-13b"), MEM.Layout(tp=1, seq=8192, batch=8), None)
    assert rc is False and e.peak > 0


def test_fp32_layout_counts_fp32_activations_and_no_shadows():
    """the planner sized fp32 runs (train.py without --bf16) as bf16.  fp32 doubles
    every activation byte and keeps no bf16 shadow; the oracle path's materialised attention
    scores are counted too."""
    a = get_preset("reference")
    bf = MEM.estimate(a, MEM.Layout(tp=1, seq=1000, batch=32))
    f32 = MEM.estimate(a, MEM.Layout(tp=1, seq=1000, batch=32, compute="fp32"))
    f32m = MEM.estimate(a, MEM.Layout(tp=1, seq=1000, batch=32, compute="fp32", materialized_attention=True))
    assert f32.parts["shadow_bf16"] == 0 and bf.parts["shadow_bf16"] > 0
    assert 1.9 < f32.parts["activations"] / bf.parts["activations"] <= 2.01
    # 12 layers x 8 heads x 32 x 1000 x 1000 fp32 probabilities kept for the backward
    assert f32m.parts["attention_scores"] == 12 * 4 * 32 * 1000 * 1000 * 8
    assert f32m.peak > f32.peak + f32m.parts["attention_scores"]
    # and the plan picks recompute / refuses on that basis
    rc, _ = MEM.plan(a, MEM.Layout(tp=1, seq=1000, batch=32, compute="fp32", materialized_attention=True),
                     f32m.peak - (1 << 30), margin_frac=0.0, margin_bytes=0)
    assert rc is True


def test_xgmi_staging_follows_the_communicator_capacity(monkeypatch):
    """xgmi_create allocates (nslots + 2) x cap + 2 x min(cap, 16 MiB) per rank."""
    assert MEM.xgmi_staging_bytes(1) == 0
    assert MEM.xgmi_staging_bytes(2, cap_mb=256) == 6 * (256 << 20) + 2 * (16 << 20)
    assert MEM.xgmi_staging_bytes(8, cap_mb=8) == 6 * (8 << 20) + 2 * (8 << 20)
    monkeypatch.setenv("DPFS_XGMI_CAP_MB", "64")
    e = MEM.estimate(get_preset("gpt2-small"), MEM.Layout(tp=2, seq=1024, batch=32))
    assert e.parts["xgmi_staging"] == 6 * (64 << 20) + 2 * (16 << 20)
