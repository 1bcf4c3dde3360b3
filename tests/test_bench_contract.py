"""bench.py driver contract on CPU/gloo: one JSON line from rank 0 with the required fields,
for a single process and for a torch.distributed.run launch with 2 ranks (TP = 2)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _env():
    e = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    return e


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("world,warmup", [(1, 1), (2, 1), (2, 4)])
def test_bench_prints_one_json_line(world, warmup):
    """warmup >= 4 at TP > 1 runs the SP on/off trial inside the warmup steps."""
    from dist_helpers import _free_port
    args = ["--gpus", str(world), "--model", "plumbing", "--steps", "2", "--warmup", str(warmup), "--seq-len", "64",
            "--batch-per-gpu", "2"]
    if world == 1:
        cmd = [sys.executable, "bench.py"] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert REQUIRED <= d.keys()
    assert d["n_gpus"] == world and d["steps"] == 2 and d["warmup"] == warmup and d["scaling"] == "weak"
    assert d["config"]["parallelism"] in (f"tp{world}", f"tp{world}+sp") and d["config"]["global_batch"] == 2 * world
    if warmup >= 4:
        assert set(d["config"]["engine_trial_ms"]) == {"sp/c2", "sp/c1"}
    if world > 1:   # pure TP is the headline here (plumbing: TP = N): one layout, labelled
        assert [L["parallelism"].split("+")[0] for L in d["layouts"]] == [f"tp{world}"]
        assert d["tp_pure"]["value"] == d["value"]
    assert d["value"] > 0 and d["higher_is_better"] is True


def test_bench_recompute_flag_and_baseline_scope():
    """--recompute reaches the model and is reported; vs_baseline is null off the GPT-2 small config."""
    cmd = [sys.executable, "bench.py", "--model", "plumbing", "--recompute", "--steps", "2", "--warmup", "1",
           "--seq-len", "64", "--batch-per-gpu", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    (d,) = _json_lines(r.stdout)
    assert d["config"]["recompute"] is True
    assert d["vs_baseline"] is None
    assert d["value"] > 0


def test_bench_tp_dp_layout():
    """--tp 2 on 4 ranks: TP pairs {0,1}, {2,3} with DP over them (the `auto` layout for
    GPT-2 small at N = 4 / 8); every replica gets its own data, the global batch stays 2 x N."""
    from dist_helpers import _free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "4", "--tp", "2", "--model", "plumbing", "--steps", "2", "--warmup", "1", "--seq-len", "64",
           "--batch-per-gpu", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    (d,) = _json_lines(r.stdout)
    assert d["config"]["parallelism"] in ("tp2dp2", "tp2dp2+sp") and d["config"]["global_batch"] == 8
    assert d["n_gpus"] == 4 and d["value"] > 0
    # the pure-TP layout (the reference's tp_size == world_size) is measured and labelled too
    labels = [L["parallelism"].split("+")[0] for L in d["layouts"]]
    assert labels == ["tp2dp2", "tp4"], labels
    assert d["tp_pure"]["parallelism"].startswith("tp4") and d["tp_pure"]["value"] > 0
    assert d["tp_pure"]["ms_per_step"] > 0


@pytest.mark.parametrize("inject", ["raise:0", "hang:3"])
def test_bench_pure_tp_failure_keeps_headline(inject):
    """A failure (exception on one rank) or a hang (one rank never arrives) in the extra pure-TP
    layout still yields exactly one JSON line with the headline numbers, tp_pure = {error}, and
    exit status 0 on every rank."""
    from dist_helpers import _free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "4", "--tp", "2", "--model", "plumbing", "--steps", "2", "--warmup", "1", "--seq-len", "64",
           "--batch-per-gpu", "2", "--pure-tp-budget-s", "25"]
    env = dict(_env(), DPFS_BENCH_INJECT=inject)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    (d,) = _json_lines(r.stdout)
    assert d["config"]["parallelism"].startswith("tp2dp2") and d["value"] > 0
    assert d["tp_pure"]["parallelism"] == "tp4" and "error" in d["tp_pure"]
    assert ("injected" in d["tp_pure"]["error"]) if inject.startswith("raise") else ("timeout" in d["tp_pure"]["error"])


def test_bench_headline_failure_is_not_a_result():
    """An exception in the TP x DP headline layout on every rank: the bench measures pure data
    parallelism for the record, but prints value = null for the requested layout (the DP
    numbers under "fallback", the failure under headline_error, no pure-TP extra) and exits
    non-zero, so a driver reading only value and the exit status cannot take it for a result."""
    from dist_helpers import _free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "4", "--tp", "2", "--model", "plumbing", "--steps", "2", "--warmup", "1", "--seq-len", "64",
           "--batch-per-gpu", "2"]
    env = dict(_env(), DPFS_BENCH_INJECT="raise_head")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0, r.stdout[-2000:] + r.stderr[-2000:]
    (d,) = _json_lines(r.stdout)
    assert d["value"] is None and d["ms_per_step"] is None and d["config"]["parallelism"] == "tp2dp2"
    assert d["fallback"]["parallelism"] == "tp1dp4" and d["fallback"]["value"] > 0
    assert d["headline_error"]["parallelism"] == "tp2dp2" and "injected" in d["headline_error"]["error"]
    assert d.get("tp_pure") is None


def test_resolve_tp():
    sys.path.insert(0, ROOT)
    from bench import resolve_tp
    assert [resolve_tp("auto", "gpt2-small", n) for n in (1, 2, 4, 8)] == [1, 2, 2, 2]
    assert [resolve_tp("auto", "llama2-7b", n) for n in (1, 2, 4, 8)] == [1, 2, 4, 8]
    assert resolve_tp("8", "gpt2-small", 8) == 8 and resolve_tp("3", "gpt2-small", 8) == 2
