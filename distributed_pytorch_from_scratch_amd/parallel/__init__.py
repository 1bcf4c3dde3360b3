from . import process_manager
from .process_manager import ProcessGroupManager, init_pgm, get_pgm
from .comm_ops import Split, Reduce, Copy, Gather, ScatterSeq, GatherSeq
from .layers import (ColumnParallelLinear, RowParallelLinear, FusedColumnParallelLinear,
                     ParallelVocabularyEmbedding, RMSNorm, LayerNorm, partition_sizes)
from .cross_entropy import vocab_parallel_cross_entropy, IGNORE_INDEX
