"""Byte-level BPE tokenizer training (reference ``train_tokenizer.py:23-67``).

HF ``tokenizers`` BPE with a ByteLevel pre-tokenizer/decoder (``add_prefix_space=True``) and the
special tokens ``<BOS>, <EOS>, <UNK>`` as ids 0, 1, 2; a round-trip self-check on a few
training texts.
"""
import argparse
import json

from ..constants import BOS_TOKEN, EOS_TOKEN, UNK_TOKEN


def train_tokenizer(texts, vocab_size: int):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE(unk_token=UNK_TOKEN))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=True)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=[BOS_TOKEN, EOS_TOKEN, UNK_TOKEN],
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    tok.train_from_iterator(texts, trainer=trainer)
    return tok


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--data_path", "-d", required=True, help="JSON from data.preprocess")
    ap.add_argument("--output", "-o", required=True)
    ap.add_argument("--vocab_size", type=int, default=1024)
    a = ap.parse_args(argv)
    texts = json.load(open(a.data_path))["train"]
    tok = train_tokenizer(texts, a.vocab_size)
    assert tok.token_to_id(BOS_TOKEN) == 0 and tok.token_to_id(EOS_TOKEN) == 1 and tok.token_to_id(UNK_TOKEN) == 2
    for t in texts[:8]:
        dec = tok.decode(tok.encode(t).ids)
        assert dec.strip() == t.strip(), (t, dec)
    tok.save(a.output)
    print(f"saved tokenizer (vocab {tok.get_vocab_size()}) -> {a.output}")


if __name__ == "__main__":
    main()
