"""End-to-end CLI (train.py / test.py), checkpoint layout + rotation + resume, TP re-sharding,
TensorBoard event files, the offline data pipeline, and fail-fast on an injected fault.
All on CPU / gloo (the reference has no test of any of these, SURVEY.md §4 gaps)."""
import glob
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=600, env=None):
    e = dict(os.environ)
    e.update({"PYTHONPATH": ROOT, "MASTER_ADDR": "127.0.0.1"})
    e.pop("WORLD_SIZE", None)
    e.pop("RANK", None)
    if env:
        e.update(env)
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=e, capture_output=True, text=True, timeout=timeout)


def _port():
    from dist_helpers import _free_port
    return str(_free_port())


def _token_json(path, V=1024, n=40, seed=0):
    g = torch.Generator().manual_seed(seed)
    data = {s: [torch.randint(3, V, (int(torch.randint(5, 40, (1,), generator=g)),), generator=g).tolist()
                for _ in range(n)] for s in ("train", "validation")}
    data["special_ids"] = {"<BOS>": 0, "<EOS>": 1, "<UNK>": 2}
    data["vocab_size"] = V
    with open(path, "w") as f:
        json.dump(data, f)


def test_train_eval_resume_cli(tmp_path):
    data = tmp_path / "tokens.json"
    _token_json(data, V=1024, n=6)
    ck = tmp_path / "ck"
    r = _run(["train.py", "--tp_size", "2", "--data_path", str(data), "--model", "plumbing", "-b", "2",
              "--max_steps", "6", "--log_interval", "2", "--save_interval", "3", "--save_dir", str(ck),
              "--reserv_last_n_ckpts", "1", "--device", "cpu", "--master_port", _port()])
    assert r.returncode == 0, r.stdout + r.stderr
    files = sorted(os.path.basename(p) for p in glob.glob(str(ck / "*.pth")))
    assert files == [f for f in files if f.startswith("tprank-")] and len(files) == 2  # rotation kept 1 per rank
    assert all("_iter-6_loss-" in f for f in files)
    sd = torch.load(str(ck / files[0]), weights_only=True)
    assert "layers.0.attn.wq.weight" in sd and "layers.0.ffn.up_proj.bias" in sd and len(sd) == 1 + 2 * 16 + 3
    ev = glob.glob(str(ck / "tprank-0" / "events.out.tfevents.*"))
    from distributed_pytorch_from_scratch_amd.utils.tb import read_scalars
    tags = {t for _, t, _ in read_scalars(ev[0])}
    assert {"train/ce_loss", "train/lr", "used_gpu_memory/tprank-0"} <= tags
    # resume from the latest checkpoint and continue to step 8
    r = _run(["train.py", "--tp_size", "2", "--data_path", str(data), "--model", "plumbing", "-b", "2",
              "--max_steps", "8", "--log_interval", "2", "--save_interval", "4", "--save_dir", str(ck),
              "--resume", "latest", "--device", "cpu", "--master_port", _port()])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "resumed from" in r.stdout and "_iter-8_" in " ".join(os.listdir(ck))
    # evaluation + greedy decode (synthetic prompts: no tokenizer file needed)
    r = _run(["test.py", "--tp_size", "2", "--ckpt_dir", str(ck), "--data_path", str(data), "--model", "plumbing",
              "--max_decode_len", "16", "--synthetic_prompts", "--device", "cpu", "--master_port", _port()])
    assert r.returncode == 0, r.stdout + r.stderr
    val = (ck / "val" / "tprank-0_val.txt").read_text()
    assert "Validation loss" in val and "Decoded" in val


def test_fault_injection_fails_fast(tmp_path):
    r = _run(["train.py", "--tp_size", "2", "--synthetic", "--model", "plumbing", "--seq_len", "32", "-b", "2",
              "--max_steps", "10", "--log_interval", "100", "--save_interval", "100", "--save_dir", str(tmp_path),
              "--fault_inject_step", "3", "--device", "cpu", "--master_port", _port()], timeout=300,
             env={"DPFS_FAULT_RANK": "1"})
    assert r.returncode != 0 and "injected fault" in (r.stdout + r.stderr)


def _get_sd(rank, world):
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    m = Transformer.from_args(ModelArgs(attn_dim=48, ffn_dim=64, num_heads=6, num_layers=1, vocab_size=50,
                                        maxlen=16, vocab_pad_to=1))
    set_seed(0)
    m.reset_parameters()
    return {k: v.clone() for k, v in m.state_dict().items()}


def test_tp_merge_split_roundtrip():
    from dist_helpers import run_distributed
    from distributed_pytorch_from_scratch_amd.utils import checkpoint as ck
    get_sd = _get_sd
    sd1 = run_distributed(get_sd, 1)[0]
    sd4 = run_distributed(get_sd, 4)
    merged = ck.merge_tp([sd4[r] for r in range(4)])
    assert merged.keys() == sd1.keys()
    for k in sd1:
        assert torch.equal(merged[k], sd1[k]), k
    split = ck.split_tp(sd1, 4, head_dim=8)
    for r in range(4):
        for k in sd1:
            assert torch.equal(split[r][k], sd4[r][k]), (r, k)


def _get_sd_balanced(rank, world):
    from distributed_pytorch_from_scratch_amd.models import Transformer, ModelArgs
    from distributed_pytorch_from_scratch_amd.utils.dist import set_seed
    m = Transformer.from_args(ModelArgs(attn_dim=48, ffn_dim=64, num_heads=6, num_layers=1, vocab_size=2000,
                                        maxlen=16, vocab_pad_to=1))
    set_seed(0)
    m.reset_parameters()
    return {k: v.clone() for k, v in m.state_dict().items()}


def test_balanced_vocab_shards_merge_split():
    """6 heads over 4 ranks (2, 2, 1, 1): the one-head ranks get larger vocab shards
    (config.vocab_partition); merge / split with those sizes round-trips exactly."""
    from dist_helpers import run_distributed
    from distributed_pytorch_from_scratch_amd.models import ModelArgs
    from distributed_pytorch_from_scratch_amd.models.config import vocab_partition
    from distributed_pytorch_from_scratch_amd.utils import checkpoint as ck
    args = ModelArgs(attn_dim=48, ffn_dim=64, num_heads=6, num_layers=1, vocab_size=2000, maxlen=16, vocab_pad_to=1)
    vs = vocab_partition(args, [2, 2, 1, 1])
    assert sum(vs) == 2000 and vs[0] < vs[2] and len(set(vs[:2])) == 1
    sd1 = run_distributed(_get_sd_balanced, 1)[0]
    sd4 = run_distributed(_get_sd_balanced, 4)
    assert [sd4[r]["embedding.weight"].size(0) for r in range(4)] == vs
    merged = ck.merge_tp([sd4[r] for r in range(4)])
    for k in sd1:
        assert torch.equal(merged[k], sd1[k]), k
    split = ck.split_tp(sd1, 4, head_dim=8, vocab_sizes=vs)
    for r in range(4):
        for k in sd1:
            assert torch.equal(split[r][k], sd4[r][k]), (r, k)


def test_data_pipeline(tmp_path):
    pytest.importorskip("tokenizers")
    raw = tmp_path / "raw.txt"
    words = ["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta", "theta"]
    g = torch.Generator().manual_seed(0)
    lines = [" ".join(words[int(i)] for i in torch.randint(0, 8, (12,), generator=g)) for _ in range(300)]
    raw.write_text("\n".join(lines))
    text, tok, toks = tmp_path / "text.json", tmp_path / "tok.json", tmp_path / "tokens.json"
    assert _run(["-m", "distributed_pytorch_from_scratch_amd.data.preprocess", "-i", str(raw), "-o", str(text)]).returncode == 0
    r = _run(["-m", "distributed_pytorch_from_scratch_amd.data.tokenizer", "-d", str(text), "-o", str(tok),
              "--vocab_size", "300"])
    assert r.returncode == 0, r.stderr
    assert _run(["-m", "distributed_pytorch_from_scratch_amd.data.pretokenize", "-d", str(text), "-t", str(tok),
                 "-o", str(toks)]).returncode == 0
    from distributed_pytorch_from_scratch_amd.data.dataset import get_dataloader
    dl = get_dataloader(str(toks), 4, split="train", maxlen=20, shuffle=False)
    b = next(iter(dl))
    ids, tgt = b["input_ids"], b["target_ids"]
    assert (ids[:, 0] == 0).all()                       # BOS first
    n0 = int((tgt[0] != -1).sum())                     # tokens + EOS
    assert tgt[0, n0 - 1] == 1 and torch.equal(ids[0, 1:n0], tgt[0, :n0 - 1])


def test_reference_tokenizer_fixture_if_present():
    """The reference ships tokenizer/tokenizer.json (BPE, vocab 1024, <BOS>/<EOS>/<UNK> = 0/1/2);
    our tokenizer tooling must load it unchanged (read-only fixture)."""
    path = "/root/reference/tokenizer/tokenizer.json"
    if not os.path.exists(path):
        pytest.skip("reference fixture not mounted")
    tokenizers = pytest.importorskip("tokenizers")
    tok = tokenizers.Tokenizer.from_file(path)
    assert tok.get_vocab_size() == 1024
    assert [tok.token_to_id(t) for t in ("<BOS>", "<EOS>", "<UNK>")] == [0, 1, 2]
    s = "Nice to meet you, it's"
    assert tok.decode(tok.encode(s).ids).strip() == s


def test_resume_reproduces_uninterrupted_run(tmp_path):
    """Stop at step 4 and resume to step 8 == train 8 steps straight: weights, optimizer,
    schedule, RNG and the data stream (same epoch order, next batch) all continue exactly."""
    data = tmp_path / "tokens.json"
    _token_json(data, V=1024, n=10)          # 5 batches per epoch at -b 2: the run crosses epochs
    a, b = tmp_path / "a", tmp_path / "b"
    common = ["train.py", "--tp_size", "2", "--data_path", str(data), "--model", "plumbing", "-b", "2",
              "--max_steps", "8", "--warmup_steps", "2", "--log_interval", "100", "--device", "cpu"]
    r = _run(common + ["--save_interval", "4", "--save_dir", str(a), "--master_port", _port()])
    assert r.returncode == 0, r.stdout + r.stderr
    os.makedirs(b)
    for f in glob.glob(str(a / "*_iter-4_*")):
        import shutil
        shutil.copy(f, b / os.path.basename(f))
    r = _run(common + ["--save_interval", "8", "--save_dir", str(b), "--resume", "latest",
                       "--master_port", _port()])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "resumed from" in r.stdout
    for rank in (0, 1):
        fa = glob.glob(str(a / f"tprank-{rank}_iter-8_*.pth"))[0]
        fb = glob.glob(str(b / f"tprank-{rank}_iter-8_*.pth"))[0]
        sa, sb = torch.load(fa, weights_only=True), torch.load(fb, weights_only=True)
        for k in sa:
            assert torch.equal(sa[k], sb[k]), (rank, k)


def test_resumable_sampler_seek():
    from distributed_pytorch_from_scratch_amd.data.dataset import SyntheticTokenDataset, _loader, seek

    class _Idx(SyntheticTokenDataset):
        def __getitem__(self, i):
            return [i + 3]

    def stream(loader, n):
        out = []
        while len(out) < n:
            for bt in loader:
                out.append(bt["input_ids"][:, 1].tolist())
                if len(out) == n:
                    break
        return out

    ds = _Idx(vocab_size=64, seq_len=4, num_samples=10)
    full = stream(_loader(ds, 3, -1, shuffle=True, seed=5), 9)      # 4 batches/epoch (last short)
    for k in (0, 2, 4, 6):
        ld = _loader(ds, 3, -1, shuffle=True, seed=5)
        seek(ld, k)
        assert stream(ld, 9 - k) == full[k:], k
    assert sorted(sum(full[:4], [])) == list(range(3, 13))         # one epoch = a permutation


def test_sidecar_loads_weights_only(tmp_path):
    """The resume sidecar (optimizer + OneCycleLR + RNG) is plain data: weights_only loads it."""
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    from distributed_pytorch_from_scratch_amd.utils import checkpoint as ck
    m = torch.nn.Linear(4, 3)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, 1e-3, total_steps=10, pct_start=0.2)
    m(torch.randn(2, 4)).sum().backward()
    opt.step()
    sched.step()
    path = ck.save_checkpoint(m, str(tmp_path), 0, 1, 1.0, opt, sched)
    side = torch.load(path + ".optim", weights_only=True)
    assert side["step"] == 1
    opt2 = FusedAdam(torch.nn.Linear(4, 3).parameters(), lr=1e-3)
    sched2 = torch.optim.lr_scheduler.OneCycleLR(opt2, 1e-3, total_steps=10, pct_start=0.2)
    st = ck.load_resume(path, opt2, sched2)
    assert st["step"] == 1 and sched2.state_dict()["last_epoch"] == 1
    s1, s2 = opt.state_dict()["state"], opt2.state_dict()["state"]
    assert all(torch.equal(s1[i]["exp_avg"], s2[i]["exp_avg"]) for i in s1)


_HB_SCRIPT = r'''
import os, sys, time
import torch.distributed as dist
import torch.multiprocessing as mp

def run(rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[1])
    dist.init_process_group("gloo", rank=rank, world_size=2)
    sys.path.insert(0, sys.argv[2])
    from distributed_pytorch_from_scratch_amd.utils.fault import Heartbeat
    hb = Heartbeat(interval_s=0.3, stale_s=2.0, abort_on_stale=True)
    hb.beat(1)
    if rank == 1:
        time.sleep(30)          # hung rank: no more heartbeats
    else:
        for s in range(200):    # healthy rank keeps beating; the watcher must abort the job
            time.sleep(0.1)
            hb.beat(s + 2)
    os._exit(0)

if __name__ == "__main__":
    mp.spawn(run, nprocs=2, join=True)
'''


def test_heartbeat_aborts_on_stale_rank(tmp_path):
    """A rank that stops beating is detected by rank 0's watcher, which aborts the job (exit
    17) long before the RCCL timeout instead of only printing a warning."""
    import time
    script = tmp_path / "hb.py"
    script.write_text(_HB_SCRIPT)
    t0 = time.time()
    r = _run([str(script), _port(), ROOT], timeout=120)
    assert r.returncode != 0, r.stdout + r.stderr
    assert "stale ranks" in (r.stdout + r.stderr)
    assert time.time() - t0 < 25


_HB_HOLD_SCRIPT = _HB_SCRIPT.replace(
    "        time.sleep(30)          # hung rank: no more heartbeats",
    "        with hb.hold(1):        # a long checkpoint save: no beats, but not a stall\n"
    "            time.sleep(5)").replace("range(200)", "range(60)")


def test_heartbeat_hold_is_not_stale(tmp_path):
    """A rank inside ``Heartbeat.hold`` (checkpoint save + barrier, evaluation) for longer
    than ``stale_s`` does not abort the job."""
    script = tmp_path / "hb_hold.py"
    script.write_text(_HB_HOLD_SCRIPT)
    r = _run([str(script), _port(), ROOT], timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "stale ranks" not in (r.stdout + r.stderr)


_HB_DEAD_IN_HOLD_SCRIPT = _HB_SCRIPT.replace(
    "hb = Heartbeat(interval_s=0.3, stale_s=2.0, abort_on_stale=True)",
    "hb = Heartbeat(interval_s=0.3, stale_s=2.0, abort_on_stale=True, max_hold_s=3.0)").replace(
    "        time.sleep(30)          # hung rank: no more heartbeats",
    "        with hb.hold(1):        # killed inside a checkpoint save: the exit beat never comes\n"
    "            time.sleep(30)")


def test_heartbeat_expired_hold_is_stale(tmp_path):
    """A rank that dies (or hangs) inside ``Heartbeat.hold`` leaves its hold marker behind: once
    the marker's deadline (``max_hold_s``) passes, the watcher flags it like any stale rank."""
    import time
    script = tmp_path / "hb_dead_hold.py"
    script.write_text(_HB_DEAD_IN_HOLD_SCRIPT)
    t0 = time.time()
    r = _run([str(script), _port(), ROOT], timeout=120)
    assert r.returncode != 0, r.stdout + r.stderr
    assert "stale ranks" in (r.stdout + r.stderr)
    assert time.time() - t0 < 25
