#!/bin/bash
# End-to-end recipe (reference recipe.sh): data -> tokenizer -> token ids -> TP=1/2/4 training
# on MI355X -> evaluation.  Every step is skipped when its output exists.
# Usage: RAW=/path/to/fineweb/000_00000.parquet WORK=./work bash recipe.sh
set -euo pipefail
RAW=${RAW:?set RAW to a FineWeb parquet shard (no download is attempted)}
WORK=${WORK:-./work}
STEPS=${STEPS:-20000}
mkdir -p "$WORK"
export HSA_ENABLE_IPC_MODE_LEGACY=0
[ -f "$WORK/text.json" ] || python -m distributed_pytorch_from_scratch_amd.data.preprocess -i "$RAW" -o "$WORK/text.json"
[ -f "$WORK/tokenizer.json" ] || python -m distributed_pytorch_from_scratch_amd.data.tokenizer -d "$WORK/text.json" -o "$WORK/tokenizer.json" --vocab_size 1024
[ -f "$WORK/tokens.json" ] || python -m distributed_pytorch_from_scratch_amd.data.pretokenize -d "$WORK/text.json" -t "$WORK/tokenizer.json" -o "$WORK/tokens.json"
for TP in 1 2 4; do
  CK="$WORK/ckpt_tp$TP"
  if [ ! -d "$CK" ]; then
    python train.py --tp_size $TP --data_path "$WORK/tokens.json" --bf16 --max_steps $STEPS --save_dir "$CK" \
      --master_port $((25555 + TP))
  fi
  [ -d "$CK/val" ] || python test.py --tp_size $TP --ckpt_dir "$CK" --data_path "$WORK/tokens.json" \
      --tokenizer_path "$WORK/tokenizer.json" --master_port $((23333 + TP))
done
