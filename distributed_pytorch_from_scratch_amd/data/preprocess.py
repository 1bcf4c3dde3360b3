"""Raw parquet -> train/validation text JSON (reference ``preprocess_data.py:10-47``).

Keeps documents of at most ``--max_chars`` characters from the ``text`` column, shuffles with
an explicit seed (the reference's split is unseeded, ``preprocess_data.py:30``) and writes
``{"train": [...], "validation": [...]}`` with a ``--val_ratio`` split.
"""
import argparse
import json
import random


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input", "-i", required=True, help="parquet file (FineWeb shard) or .txt/.jsonl")
    ap.add_argument("--output", "-o", required=True)
    ap.add_argument("--max_chars", type=int, default=2000)
    ap.add_argument("--val_ratio", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    if a.input.endswith(".parquet"):
        import pandas as pd
        texts = pd.read_parquet(a.input, columns=["text"])["text"].tolist()
    elif a.input.endswith(".jsonl"):
        texts = [json.loads(l)["text"] for l in open(a.input)]
    else:
        texts = [l.rstrip("\n") for l in open(a.input) if l.strip()]
    texts = [t for t in texts if len(t) <= a.max_chars]
    random.Random(a.seed).shuffle(texts)
    n_val = max(1, int(len(texts) * a.val_ratio))
    with open(a.output, "w") as f:
        json.dump({"train": texts[n_val:], "validation": texts[:n_val]}, f)
    print(f"wrote {len(texts) - n_val} train / {n_val} validation docs -> {a.output}")


if __name__ == "__main__":
    main()
