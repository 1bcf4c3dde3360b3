"""Rehearsal of the driver's 8-GPU bench on one MI355X: ``bench.py --gpus 8`` under
``torch.distributed.run`` with 8 ranks sharing the GPU (gloo bootstrap; RCCL refuses two ranks
on one device), the ``auto`` TP transport decision enabled on gloo
(``DPFS_TP_COMM_AUTO_ANY_BACKEND=1``: xGMI kernels and the relayed TP = 2 exchange are built,
validated and timed), and a reduced model (1 layer, seq 128) so it fits the test time limit.

It runs the same code as the driver's run: the headline ``tp2dp4`` layout with the relay
candidate, then the extra pure ``tp8`` layout (12 heads over 8 ranks: 2 / 1 per rank) over the
xGMI kernels, both reported in ONE JSON line with their transport decisions.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_bench_8_ranks_on_one_gpu():
    from dist_helpers import _free_port
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", DPFS_BACKEND="gloo", DPFS_TP_COMM="auto",
               DPFS_TP_COMM_AUTO_ANY_BACKEND="1", DPFS_GEMM_BACKEND="ours", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "8", "--layers", "1", "--seq-len", "128", "--batch-per-gpu", "2", "--steps", "2",
           "--warmup", "2", "--pure-tp-budget-s", "120"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = lines[0]
    if os.environ.get("DPFS_REHEARSAL_OUT"):     # keep the line (profiles/ record of the rehearsal)
        with open(os.environ["DPFS_REHEARSAL_OUT"], "w") as f:
            f.write(json.dumps(d) + "\n")
    assert d["n_gpus"] == 8 and d["value"] > 0
    assert d["config"]["parallelism"].startswith("tp2dp4")
    assert [L["parallelism"].split("+")[0] for L in d["layouts"]] == ["tp2dp4", "tp8"], d["layouts"]
    head, pure = d["layouts"]
    assert "error" not in d["tp_pure"], d["tp_pure"]
    assert d["tp_pure"]["value"] > 0
    # both layouts made (and report) a transport decision per op
    for L in (head, pure):
        assert L["tp_comm"] is not None and "transport" in L["tp_comm"], L
    assert "relay_ms" in head["tp_comm"]["all_reduce"]          # the relay was a candidate at tp2dp4
    assert "xgmi_blocks" in pure["tp_comm"]["all_reduce"]       # the xGMI kernels at tp8
