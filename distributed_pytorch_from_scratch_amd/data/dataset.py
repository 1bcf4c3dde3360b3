"""Token datasets, collate function and loaders.

Reference parity: ``dataset.py:12-68`` — the pre-tokenised JSON format
``{"train": [[ids]], "validation": [[ids]], "special_ids": {...}, "vocab_size": int}``
(written by ``pre_tokenize.py``), truncation to ``maxlen - 1`` tokens, and the collate rule:

    input  = [BOS, t_0 .. t_{n-1}, EOS, EOS, ...]      (length max_len + 1)
    target = [t_0 .. t_{n-1}, EOS, -1, -1, ...]        (IGNORE_INDEX padding)
    position_ids = arange(max_len + 1)

Differences: the dataset is named for what it is (``TokenJsonDataset``; the reference's
``ShakespeareDataset`` alias is kept), the truncation warning is emitted once instead of
per sample, the DataLoader is seeded explicitly (every TP rank must see the same batch —
the reference relies on identical global seeds), and there is a ``SyntheticTokenDataset``
for benchmarks / CI (no dataset download on the target machines).
"""
from __future__ import annotations

import json
import os
import warnings
from functools import partial
from typing import Dict, List, Optional

import torch
from torch.utils.data import DataLoader, Dataset, Sampler

from ..constants import BOS_TOKEN, EOS_TOKEN, UNK_TOKEN, IGNORE_INDEX


class TokenJsonDataset(Dataset):
    def __init__(self, data_path: str, split: str, maxlen: int):
        assert split in ("train", "validation"), f"split must be train/validation, got {split}"
        assert os.path.exists(data_path), data_path
        with open(data_path, "r") as f:
            data = json.load(f)
        if split not in data:
            raise ValueError(f"Split {split} not found in {data_path}; available: {list(data.keys())}")
        self.samples: List[List[int]] = data[split]
        self.maxlen = maxlen
        self.split = split
        sp = data["special_ids"]
        self.bos, self.eos, self.unk = sp[BOS_TOKEN], sp[EOS_TOKEN], sp[UNK_TOKEN]
        self.vocab_size = int(data["vocab_size"])
        self._warned = False

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, idx: int) -> List[int]:
        toks = self.samples[idx]
        if len(toks) > self.maxlen - 1:   # reserve one position for BOS/EOS
            if not self._warned:
                warnings.warn(f"sequences longer than maxlen-1={self.maxlen - 1} are truncated")
                self._warned = True
            toks = toks[: self.maxlen - 1]
        return toks


ShakespeareDataset = TokenJsonDataset  # reference name


class SyntheticTokenDataset(Dataset):
    """Deterministic random token sequences (uniform ids in [3, vocab)), fixed length."""

    def __init__(self, vocab_size: int, seq_len: int, num_samples: int = 1 << 20, seed: int = 0,
                 bos: int = 0, eos: int = 1, unk: int = 2):
        self.vocab_size, self.seq_len, self.n, self.seed = vocab_size, seq_len, num_samples, seed
        self.bos, self.eos, self.unk = bos, eos, unk

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, idx: int) -> List[int]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        return torch.randint(3, self.vocab_size, (self.seq_len - 1,), generator=g).tolist()


def collate_fn(batch: List[List[int]], bos: int, eos: int, ignore_idx: int) -> Dict[str, torch.Tensor]:
    max_len = max(len(x) for x in batch)
    n = len(batch)
    input_ids = torch.full((n, max_len + 1), eos, dtype=torch.long)
    target_ids = torch.full((n, max_len + 1), ignore_idx, dtype=torch.long)
    for i, b in enumerate(batch):
        t = torch.tensor(b, dtype=torch.long)
        input_ids[i, 0] = bos
        input_ids[i, 1:len(b) + 1] = t
        target_ids[i, :len(b)] = t
        target_ids[i, len(b)] = eos
    position_ids = torch.arange(max_len + 1).unsqueeze(0).repeat(n, 1)
    return {"input_ids": input_ids, "target_ids": target_ids, "position_ids": position_ids}


class ResumableSampler(Sampler):
    """Epoch-indexed sample order that can start mid-epoch (extension: the reference restarts
    its DataLoader from scratch, so it cannot resume a run at the batch it stopped at).

    Epoch ``e`` visits ``randperm(n)`` drawn from a generator seeded ``seed + e`` (or
    ``arange(n)`` without shuffling), so any epoch's order is reproducible without replaying
    the earlier ones; ``set_epoch(e, skip)`` makes the next iteration start ``skip`` samples in.
    """

    def __init__(self, n: int, shuffle: bool, seed: int):
        self.n, self.shuffle, self.seed = n, shuffle, seed
        self.epoch, self.skip = 0, 0

    def set_epoch(self, epoch: int, skip: int = 0) -> None:
        self.epoch, self.skip = epoch, skip

    def __len__(self) -> int:
        return self.n - self.skip

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g)
        else:
            order = torch.arange(self.n)
        skip, self.skip = self.skip, 0
        self.epoch += 1
        return iter(order[skip:].tolist())


def _loader(ds, batch_size, ignore_idx, shuffle, seed, num_workers=0, drop_last=False):
    sampler = ResumableSampler(len(ds), shuffle, seed)
    # The generator only feeds DataLoader's per-iteration base seed, keeping the global RNG
    # untouched by data loading.
    g = torch.Generator()
    g.manual_seed(seed)
    return DataLoader(ds, batch_size=batch_size, sampler=sampler, generator=g,
                      collate_fn=partial(collate_fn, bos=ds.bos, eos=ds.eos, ignore_idx=ignore_idx),
                      num_workers=num_workers, pin_memory=torch.cuda.is_available(), drop_last=drop_last)


def resume_position(loader: DataLoader, step: int):
    """(epoch, batches into that epoch) after ``step`` optimizer steps with one batch per step."""
    n = loader.sampler.n
    per_epoch = n // loader.batch_size if loader.drop_last else -(-n // loader.batch_size)
    per_epoch = max(1, per_epoch)
    return step // per_epoch, step % per_epoch


def seek(loader: DataLoader, step: int) -> int:
    """Position ``loader`` so its next iteration yields the batch of optimizer step ``step + 1``;
    returns the epoch that iteration belongs to."""
    epoch, k = resume_position(loader, step)
    loader.sampler.set_epoch(epoch, k * loader.batch_size)
    return epoch


def get_dataloader(data_path: str, batch_size: int, ignore_idx: int = IGNORE_INDEX, split: str = "train",
                   maxlen: int = 1000, shuffle: bool = True, seed: int = 0, num_workers: int = 0) -> DataLoader:
    """Reference signature (``dataset.py:58``) + an explicit shuffle seed."""
    return _loader(TokenJsonDataset(data_path, split, maxlen), batch_size, ignore_idx, shuffle, seed, num_workers)


def get_synthetic_dataloader(vocab_size: int, seq_len: int, batch_size: int, seed: int = 0,
                             num_samples: int = 1 << 20, ignore_idx: int = IGNORE_INDEX) -> DataLoader:
    ds = SyntheticTokenDataset(vocab_size, seq_len, num_samples, seed)
    return _loader(ds, batch_size, ignore_idx, shuffle=False, seed=seed, drop_last=True)
