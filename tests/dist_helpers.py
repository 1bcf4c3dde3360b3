"""Multi-process test harness (gloo on CPU, one process per rank).

Unlike the reference's ``mp.spawn`` + ``unittest.TextTestRunner`` scripts (whose failures
never reach the exit code), any exception in any rank fails the pytest case
with that rank's traceback.
"""
import io
import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world_size, port, fn, args, tp_size, backend, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        torch.set_num_threads(max(1, 8 // world_size))
        from distributed_pytorch_from_scratch_amd.utils.dist import init_dist_env, destroy_dist_env
        init_dist_env(rank=rank, tp_size=tp_size or world_size, world_size=world_size,
                      backend=backend)
        res = fn(rank, world_size, *args)
        buf = io.BytesIO()
        torch.save(res, buf)   # plain bytes: no shared-memory handles outliving the worker
        q.put((rank, "ok", buf.getvalue()))
        destroy_dist_env()
    except BaseException:
        q.put((rank, "err", traceback.format_exc()))


def run_distributed(fn, world_size, *args, tp_size=None, backend="gloo", timeout=300):
    """Run ``fn(rank, world_size, *args)`` on ``world_size`` ranks; return {rank: result}."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, fn, args, tp_size, backend, q))
             for r in range(world_size)]
    for p in procs:
        p.start()
    results, errors = {}, []
    for _ in range(world_size):
        try:
            rank, status, payload = q.get(timeout=timeout)
        except Exception as e:
            errors.append(f"no result from a rank within {timeout}s ({e!r})")
            break
        if status == "ok":
            import torch
            results[rank] = torch.load(io.BytesIO(payload), weights_only=False)
        else:
            errors.append(f"[rank {rank}]\n{payload}")
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    if errors:
        raise AssertionError("\n".join(errors))
    return results
