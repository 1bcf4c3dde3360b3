#!/usr/bin/env python
"""``python train.py --tp_size N --data_path D [--bf16]`` (reference CLI; see
distributed_pytorch_from_scratch_amd/train.py for all flags)."""
from distributed_pytorch_from_scratch_amd.train import main

if __name__ == "__main__":
    main()
