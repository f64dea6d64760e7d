from .tokenizer import BPETokenizer, ByteTokenizer, Llama2Tokenizer, Llama3Tokenizer, build_tokenizer  # noqa: F401
from .datasets import DatasetPT, InstructionDataset, custom_collate_fn, format_input  # noqa: F401
from .loaders import DataloaderPT, DataloaderIF  # noqa: F401
from .synthetic import make_alpaca_json, make_gutenberg_corpus  # noqa: F401
