from .base import BaseLM, LocalEngine, RunCtx  # noqa: F401
from .gpt2 import GPTModel  # noqa: F401
from .llama import LlamaModel, Llama2Model, Llama3Model, RMSNorm  # noqa: F401
from .lora import LoRALayer, LinearWithLoRA, replace_linear_with_lora  # noqa: F401


def build_model(cfg, use_actv_ckpt=False, device=None):
    """GPT-2 or Llama model for a :class:`~building_llm_from_scratch_amd.config.ModelConfig`."""
    if cfg.family == "gpt2":
        return GPTModel(cfg, use_actv_ckpt, device=device)
    return LlamaModel(cfg, use_actv_ckpt, device=device)
