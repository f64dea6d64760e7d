"""MI355X-native GPT-2 / Llama training framework (gfx950, PyTorch-ROCm + HIP + RCCL).

Capabilities of chemphenoms/Building_LLM_from_scratch, re-designed for MI355X:
see README.md and SURVEY.md.
"""
__version__ = "0.1.0"

from .config import ModelConfig, get_config, debug_config  # noqa: F401
