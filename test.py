#!/usr/bin/env python
"""``python test.py --tp_size N --ckpt_dir C --data_path D --tokenizer_path T`` — validation loss
over checkpoints + greedy decoding (reference CLI; see
distributed_pytorch_from_scratch_amd/evaluate.py)."""
from distributed_pytorch_from_scratch_amd.evaluate import main

if __name__ == "__main__":
    main()
