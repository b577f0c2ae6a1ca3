"""Model families: Llama-style decoders (llama.py), BERT/BGE encoders (bert.py), configs (config.py)."""
from .config import DECODERS, ENCODERS, DecoderConfig, EncoderConfig, decoder_config, encoder_config  # noqa: F401
