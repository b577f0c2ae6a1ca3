"""Local generation engine: paged-KV continuous batching on one MI355X per process."""
from .sampling import SamplingParams  # noqa: F401
from .tokenizer import ByteTokenizer, IncrementalDecoder  # noqa: F401
