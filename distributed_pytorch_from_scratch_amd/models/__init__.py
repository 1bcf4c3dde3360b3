from .config import ModelArgs, ModelArgumments, PRESETS, get_preset
from .transformer import Transformer, DecoderLayer, Attention, FFN, build_model
from .rope import rotate_half, apply_rotary_pos_emb, get_cos_sin
