"""Text JSON -> token-id JSON consumed by ``data.dataset`` (reference ``pre_tokenize.py:20-52``):
``{"train": [[ids]], "validation": [[ids]], "special_ids": {"<BOS>":0,...}, "vocab_size": V}``."""
import argparse
import json

from ..constants import BOS_TOKEN, EOS_TOKEN, UNK_TOKEN


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--data_path", "-d", required=True)
    ap.add_argument("--tokenizer_path", "-t", required=True)
    ap.add_argument("--output", "-o", required=True)
    a = ap.parse_args(argv)
    from tokenizers import Tokenizer
    tok = Tokenizer.from_file(a.tokenizer_path)
    data = json.load(open(a.data_path))
    out = {}
    for split in ("train", "validation"):
        out[split] = [e.ids for e in tok.encode_batch(data[split])]
    out["special_ids"] = {t: tok.token_to_id(t) for t in (BOS_TOKEN, EOS_TOKEN, UNK_TOKEN)}
    out["vocab_size"] = tok.get_vocab_size()
    with open(a.output, "w") as f:
        json.dump(out, f)
    print(f"tokenized {len(out['train'])} train / {len(out['validation'])} validation -> {a.output}")


if __name__ == "__main__":
    main()
