"""Per-rank checkpoints in the reference layout, rotation, resume and TP re-sharding.

Reference parity (``train.py:121-133``, ``test.py:49-55,94-95``):

* one file per TP rank per save: ``{save_dir}/tprank-{r}_iter-{step}_loss-{cumavg:.4f}.pth``
  containing ``model.state_dict()`` only (196 keys at L=12; the fused QKV / gate|up weights are
  presented as the reference's separate ``wq/wk/wv`` / ``gate_proj/up_proj`` keys);
* keep-last-N rotation ordered by the parsed iteration;
* discovery by glob ``tprank-{r}_iter-*_loss-*.pth`` sorted by iteration.

Extensions: an optional sidecar ``...pth.optim`` with optimizer + scheduler + RNG + step for
real resume (the reference cannot resume), files written atomically (tmp + rename), loads use
``weights_only=True``, and ``merge_tp`` / ``split_tp`` convert between TP degrees (possible
because every sharded tensor is a contiguous slice of the full reference-initialised matrix).
With DP > 1 only DP rank 0 of each TP group writes (replicas are identical).
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, List, Optional, Sequence

import torch

_PAT = re.compile(r"tprank-(\d+)_iter-(\d+)_loss-(.+?)\.pth$")


def ckpt_name(tp_rank: int, step: int, loss: float) -> str:
    return f"tprank-{tp_rank}_iter-{step}_loss-{loss:.4f}.pth"


def list_checkpoints(ckpt_dir: str, tp_rank: int) -> List[str]:
    paths = glob.glob(os.path.join(ckpt_dir, f"tprank-{tp_rank}_iter-*_loss-*.pth"))
    return sorted(paths, key=lambda p: int(_PAT.search(os.path.basename(p)).group(2)))


def parse_iter(path: str) -> int:
    return int(_PAT.search(os.path.basename(path)).group(2))


def _atomic_save(obj, path: str):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_checkpoint(model: torch.nn.Module, save_dir: str, tp_rank: int, step: int, loss: float,
                    optimizer=None, scheduler=None, extra: Optional[dict] = None,
                    keep_last_n: int = -1) -> str:
    os.makedirs(save_dir, exist_ok=True)
    path = os.path.join(save_dir, ckpt_name(tp_rank, step, loss))
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    _atomic_save(sd, path)
    if optimizer is not None:
        side = {"optimizer": optimizer.state_dict(), "step": step,
                "scheduler": scheduler.state_dict() if scheduler is not None else None,
                "rng_cpu": torch.get_rng_state(),
                "rng_cuda": torch.cuda.get_rng_state() if torch.cuda.is_available() else None,
                "extra": extra or {}}
        _atomic_save(side, path + ".optim")
    if keep_last_n > 0:
        for old in list_checkpoints(save_dir, tp_rank)[:-keep_last_n]:
            os.remove(old)
            if os.path.exists(old + ".optim"):
                os.remove(old + ".optim")
    return path


def load_model(model: torch.nn.Module, path: str, dtype: Optional[torch.dtype] = None,
               strict: bool = True) -> None:
    """Load a per-rank state dict (``weights_only=True``); ``dtype`` casts like the reference's
    ``load_ckpt`` (``test.py:49-55``)."""
    dev = next(model.parameters()).device
    sd = torch.load(path, map_location=dev, weights_only=True)
    if dtype is not None:
        sd = {k: v.to(dtype) for k, v in sd.items()}
        model.to(dtype)
    model.load_state_dict(sd, strict=strict)


def load_resume(path: str, optimizer=None, scheduler=None) -> Optional[dict]:
    side = path + ".optim"
    if not os.path.exists(side):
        return None
    # Everything in the sidecar is plain data (state dicts, ByteTensor RNG states, ints, dicts),
    # so the weights-only unpickler loads it; nothing in the file can execute code.
    st = torch.load(side, map_location="cpu", weights_only=True)
    if optimizer is not None:
        optimizer.load_state_dict(st["optimizer"])
    if scheduler is not None and st.get("scheduler") is not None:
        scheduler.load_state_dict(st["scheduler"])
    if st.get("rng_cpu") is not None:
        torch.set_rng_state(st["rng_cpu"])
    if st.get("rng_cuda") is not None and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["rng_cuda"])
    return st


# ------------------------------------------------------------------ TP re-sharding ----
# Shard axis of every reference key: 0 = rows (column-parallel / vocab), 1 = cols (row-parallel),
# None = replicated.
def shard_dim(key: str) -> Optional[int]:
    if key.endswith("scale") or key.endswith("wo.bias") or key.endswith("down_proj.bias") or \
            ".norm" in key or key.startswith("norm."):
        return None
    if key.endswith("wo.weight") or key.endswith("down_proj.weight"):
        return 1
    return 0


def merge_tp(shards: Sequence[Dict[str, torch.Tensor]]) -> Dict[str, torch.Tensor]:
    """Concatenate TP shards (ordered by tp rank) into a TP=1 state dict."""
    out = {}
    for k in shards[0]:
        d = shard_dim(k)
        out[k] = shards[0][k].clone() if d is None else torch.cat([s[k] for s in shards], dim=d)
    return out


def split_tp(full: Dict[str, torch.Tensor], n: int, head_dim: Optional[int] = None,
             vocab_sizes: Optional[Sequence[int]] = None) -> List[Dict[str, torch.Tensor]]:
    """Split a TP=1 state dict into ``n`` shards using the framework's partition rules
    (heads whole when ``head_dim`` is given; vocab shards = ``vocab_sizes`` — e.g.
    ``models.config.vocab_partition`` for a model built with an uneven head split — or the
    reference ranges, remainder on the last rank)."""
    from ..parallel.layers import partition_sizes
    outs = [dict() for _ in range(n)]
    for k, v in full.items():
        d = shard_dim(k)
        if d is None:
            for o in outs:
                o[k] = v.clone()
            continue
        total = v.size(d)
        if k.startswith("embedding") or k.startswith("lm_head"):
            if vocab_sizes is not None:
                sizes = list(vocab_sizes)
            else:
                per = total // n
                sizes = [per] * (n - 1) + [total - per * (n - 1)]
        elif head_dim and (".attn." in k):
            sizes = partition_sizes(total, n, head_dim)
        else:
            sizes = partition_sizes(total, n)
        for r, part in enumerate(torch.split(v, sizes, dim=d)):
            outs[r][k] = part.clone()
    return outs
