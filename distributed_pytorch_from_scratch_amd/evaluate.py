"""Evaluation + greedy decoding entrypoint (the reference's ``test.py``).

Reference parity: ``test.py:23-172`` — CLI ``--master_addr --master_port --tp_size
--data_path/-d --tokenizer_path/-t --ckpt_dir --use_vallina_impl --max_decode_len
--random_seed``; for every ``tprank-{r}_iter-*_loss-*.pth`` of this rank (sorted by iteration)
the validation loss (batch 1, bf16) is written to ``{ckpt_dir}/val/tprank-{r}_val.txt`` and TB
``val/loss``; then the last checkpoint greedily continues 8 fixed prompts until EOS or
``max_decode_len``.

Fixed reference bugs: the decode loads ``ckpt_paths[-1]`` (the reference
indexes the last *character* of a path string, ``test.py:124``), and the embedding no longer
mutates the token buffer, so TP>1 decoding is correct.  Extensions: ``--synthetic_prompts``
(token-id prompts when no tokenizer file is available) and the vocab-parallel loss.
"""
from __future__ import annotations

import os
import re
from argparse import ArgumentParser

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .constants import BOS_TOKEN, EOS_TOKEN, IGNORE_INDEX
from .data.dataset import get_dataloader
from .models import Transformer, get_preset
from .parallel import process_manager as pm
from .utils import checkpoint as ck
from .utils.dist import destroy_dist_env, init_dist_env, set_seed
from .utils.tb import SummaryWriter

PROMPTS = [
    "Nice to meet you, it's",
    "Great empire never falls, it only",
    "Your majesty, it's my duty ",
    "I shall be glad ",
    "What a glory to ",
    "Shame for the weak, it's",
    "The brave man ne",
    "Poor old man, it's",
]


def _backend(use_cuda: bool) -> str:
    """RCCL on GPUs; ``DPFS_BACKEND=gloo`` runs several ranks on one GPU (the TP collectives
    then go through ``DPFS_TP_COMM``'s transports, e.g. the xGMI kernels)."""
    return os.environ.get("DPFS_BACKEND") or ("nccl" if use_cuda else "gloo")


def get_test_args(argv=None):
    p = ArgumentParser()
    g = p.add_argument_group("distributed")
    g.add_argument("--master_addr", type=str, default="127.0.0.1")
    g.add_argument("--master_port", type=str, default="23333")
    g.add_argument("--tp_size", type=int, default=2)
    g = p.add_argument_group("data")
    g.add_argument("--data_path", "-d", type=str, required=True)
    g.add_argument("--tokenizer_path", "-t", type=str, default=None)
    g = p.add_argument_group("model")
    g.add_argument("--use_vallina_impl", action="store_true")
    g.add_argument("--model", type=str, default="reference")
    p.add_argument("--ckpt_dir", type=str, required=True)
    g = p.add_argument_group("decode")
    g.add_argument("--max_decode_len", type=int, default=128)
    g.add_argument("--synthetic_prompts", action="store_true")
    g.add_argument("--no_kv_cache", action="store_true", help="re-run the full prefix per token (reference)")
    g = p.add_argument_group("other")
    g.add_argument("--random_seed", type=int, default=0)
    g.add_argument("--device", type=str, default=None)
    return p.parse_args(argv)


@torch.inference_mode()
def calc_loss(model: Transformer, dataloader, dev) -> float:
    total, n = 0.0, 0
    for batch in dataloader:
        ids = batch["input_ids"].to(dev)
        tgt = batch["target_ids"].to(dev)
        pos = batch["position_ids"].to(dev)
        logits = model(ids, pos)
        loss = F.cross_entropy(logits.float().reshape(-1, logits.size(-1)), tgt.reshape(-1),
                               ignore_index=IGNORE_INDEX, reduction="mean")
        total += float(loss.item())
        n += 1
    return total / max(1, n)


@torch.inference_mode()
def greedy_decode(model: Transformer, prompt_ids, bos: int, eos: int, max_len: int, dev, kv_cache: bool = True):
    """Greedy continuation of ``[bos] + prompt`` until EOS or ``max_len + 1`` tokens (the
    reference's stopping rule, ``test.py:144-150``); returns the ids after BOS without EOS.
    ``kv_cache`` decodes one token per step against cached keys/values
    (``models/generation.py``); ``False`` re-runs the whole prefix per token like the reference."""
    if kv_cache:
        from .models.generation import generate
        n0 = 1 + len(prompt_ids)
        tokens = torch.tensor([bos] + list(prompt_ids), dtype=torch.long, device=dev).view(1, -1)
        out = generate(model, tokens, max_new_tokens=max(1, max_len + 1 - n0), eos_id=eos)[0]
        out = out[1:]
        if out and out[-1] == eos and len(out) > len(prompt_ids):
            out = out[:-1]
        return out
    tokens = torch.tensor([bos] + list(prompt_ids), dtype=torch.long, device=dev).view(1, -1)
    while True:
        pos = torch.arange(tokens.size(1), device=dev).unsqueeze(0)
        logits = model(tokens, pos)[0, -1]
        nxt = int(logits.argmax(-1).item())
        tokens = torch.cat([tokens, torch.tensor([[nxt]], device=dev)], dim=1)
        if nxt == eos or tokens.size(1) > max_len:
            out = tokens[0, 1:]
            if nxt == eos:
                out = out[:-1]
            return out.tolist()


def test(rank, args):
    set_seed(args.random_seed)
    use_cuda = (args.device or ("cuda" if torch.cuda.is_available() else "cpu")) == "cuda"
    p = init_dist_env(args, rank, world_size=args.tp_size, backend=_backend(use_cuda))
    dev = torch.device("cuda", torch.cuda.current_device()) if use_cuda else torch.device("cpu")
    margs = get_preset(args.model)
    model = Transformer.from_args(margs).to(dev)
    model.reset_parameters()
    model.eval()
    dtype = torch.bfloat16 if use_cuda else torch.float32
    model.set_compute_dtype(dtype)

    paths = ck.list_checkpoints(args.ckpt_dir, p.tp_rank)
    if not paths:
        raise ValueError(f"[TP Rank {p.tp_rank}]: No checkpoints found in {args.ckpt_dir}")
    print(f"[TP Rank {p.tp_rank}]: Found {len(paths)} checkpoints.", flush=True)

    loader = get_dataloader(args.data_path, 1, IGNORE_INDEX, split="validation", maxlen=margs.maxlen,
                            shuffle=False)
    save_path = os.path.join(args.ckpt_dir, "val", f"tprank-{p.tp_rank}_val.txt")
    os.makedirs(os.path.dirname(save_path), exist_ok=True)
    writer = SummaryWriter(os.path.join(args.ckpt_dir, f"tprank-{p.tp_rank}"))
    results = []
    with open(save_path, "a") as f:
        f.write("Ckpt -> Validation loss\n")
        for path in paths:
            it = ck.parse_iter(path)
            ck.load_model(model, path)   # fp32 master weights; bf16 compute via the kernels
            loss = calc_loss(model, loader, dev)
            f.write(f"{path} -> {loss:.4f}\n")
            writer.add_scalar("val/loss", loss, it)
            results.append((it, loss))
    writer.close()

    ck.load_model(model, paths[-1])
    ds = loader.dataset
    decoded = []
    if args.synthetic_prompts or not args.tokenizer_path:
        for i in range(4):
            g = torch.Generator().manual_seed(i)
            ids = torch.randint(3, margs.vocab_size, (8,), generator=g).tolist()
            out = greedy_decode(model, ids, ds.bos, ds.eos, args.max_decode_len, dev, not args.no_kv_cache)
            assert out[:len(ids)] == ids
            decoded.append((str(ids), str(out[len(ids):])))
    else:
        from tokenizers import Tokenizer
        tok = Tokenizer.from_file(args.tokenizer_path)
        assert tok.token_to_id(BOS_TOKEN) == ds.bos and tok.token_to_id(EOS_TOKEN) == ds.eos
        for t in PROMPTS:
            t = t.strip()
            ids = tok.encode(t).ids
            out = greedy_decode(model, ids, ds.bos, ds.eos, args.max_decode_len, dev, not args.no_kv_cache)
            text = tok.decode(out).strip()
            decoded.append((t, text[len(t):] if text.startswith(t) else text))
    with open(save_path, "a") as fp:
        print("\n\nInput texts -> Decoded texts", file=fp)
        for a_, b_ in decoded:
            print(f"{a_} -> {b_}", file=fp)
            if p.tp_rank == 0:
                print(f"{a_} -> {b_}", flush=True)
    dist.barrier()
    destroy_dist_env()
    return results


def main(argv=None):
    args = get_test_args(argv)
    import torch.multiprocessing as mp
    os.environ.setdefault("MASTER_ADDR", args.master_addr)
    mp.spawn(test, args=(args,), nprocs=args.tp_size, join=True)


if __name__ == "__main__":
    main()
