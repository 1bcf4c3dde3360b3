from .config import ModelArgs, ModelArgumments, PRESETS, get_preset
from .transformer import Transformer, DecoderLayer, Attention, FFN, build_model
