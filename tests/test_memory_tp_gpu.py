"""HBM planner at TP 2 / 4 / 8: rank r's exact shards and per-rank
batch are built on ONE GPU (tools/tp_sim.py, every collective a no-op, so the xGMI staging term
is left out of the estimate) for the bench's multi-GPU layouts (SP, two ping-pong chunks, and
one chunk without SP), and the planner's per-rank estimate (utils/memory.py) must be within
10 % of ``torch.cuda.max_memory_allocated`` of the steady-state step."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("tp,rank", [(2, 0), (4, 0), (8, 0), (8, 7)])
def test_planner_per_rank_estimate_at_tp(tp, rank):
    cmd = [sys.executable, os.path.join(ROOT, "tools", "tp_sim.py"), "--tp", str(tp), "--rank", str(rank),
           "--batch-per-gpu", "8", "--steps", "1", "--configs", "sp:2,nosp:1", "--mem-check"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 2, out.stdout
    for ln in lines:
        print(ln)
        assert 0.9 <= ln["est_over_measured"] <= 1.1, ln
