from .tokenizer import BPETokenizer, ByteTokenizer, Llama2Tokenizer, Llama3Tokenizer, build_tokenizer  # noqa: F401
from .datasets import (DatasetPT, InstructionDataset, InstructionDatasetPhi, custom_collate_fn,  # noqa: F401
                       format_input, format_input_phi)
from .loaders import DataloaderPT, DataloaderIF  # noqa: F401
from .synthetic import make_alpaca_json, make_gutenberg_corpus  # noqa: F401
