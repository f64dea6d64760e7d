"""Mixed-precision policies (reference ``datautils/mixed_precision.py:10-46``).

The reference defines torch-FSDP ``MixedPrecision(param, reduce, buffer)`` objects and the
builder imports names that do not exist (SURVEY §2.8 defect 2), so ``--use_fsdp`` never runs
there.  Here a policy is a plain frozen record consumed by our own engines:

* ``param_dtype``  — storage/compute dtype of the parameters the kernels see (bf16/fp16 run on
  the CDNA4 MFMA path; fp32 runs the fp32 fallback kernels).
* ``reduce_dtype`` — dtype of the gradient collectives (RCCL reduce-scatter / all-reduce).
  Gradients are produced in ``param_dtype``; a different reduce dtype costs one cast.
* ``buffer_dtype`` — non-parameter buffers.  Our models keep their RoPE tables / masks in fp32
  internally (never communicated), so this only sets the dtype of the parity state-dict
  entries (``att.cos`` / ``att.sin``).
* ``master_dtype`` — the optimizer's master weights and AdamW moments.  Always fp32 when the
  params are 16-bit (the reference's pure-bf16 AdamW loses updates below bf16 resolution).
* ``loss_scaling`` — fp16 needs dynamic loss scaling (the Trainer's DynamicLossScaler).

``bf16_hybrid_policy`` (fp32 params, bf16 reduce) keeps fp32 parameters and halves the
gradient traffic.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict

import torch


@dataclass(frozen=True)
class MixedPrecision:
    param_dtype: torch.dtype = torch.float32
    reduce_dtype: torch.dtype = torch.float32
    buffer_dtype: torch.dtype = torch.float32
    master_dtype: torch.dtype = torch.float32

    @property
    def loss_scaling(self) -> bool:
        return self.param_dtype == torch.float16

    def describe(self) -> str:
        n = lambda d: str(d).replace("torch.", "")  # noqa: E731
        return (f"MixedPrecision(param_dtype={n(self.param_dtype)}, reduce_dtype={n(self.reduce_dtype)}, "
                f"buffer_dtype={n(self.buffer_dtype)}, master_dtype={n(self.master_dtype)}, "
                f"loss_scaling={self.loss_scaling})")

    __str__ = describe


fp16_policy = MixedPrecision(torch.float16, torch.float16, torch.float16)
bf16_policy = MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16)
bf16_hybrid_policy = MixedPrecision(torch.float32, torch.bfloat16, torch.bfloat16)
fp32_policy = MixedPrecision(torch.float32, torch.float32, torch.float32)

mixed_precision_policies: Dict[str, MixedPrecision] = {
    "fp16": fp16_policy,
    "bf16": bf16_policy,
    "bf16_hybrid": bf16_hybrid_policy,
    "fp32": fp32_policy,
}

# the reference builder's (non-existent) import names, provided so that code written against
# the intended API resolves (build_components.py:166)
fpSixteen = fp16_policy
bfSixteen = bf16_policy


def get_policy(name_or_policy) -> MixedPrecision:
    if isinstance(name_or_policy, MixedPrecision):
        return name_or_policy
    try:
        return mixed_precision_policies[str(name_or_policy)]
    except KeyError:
        raise ValueError(f"unknown mixed-precision policy '{name_or_policy}' "
                         f"(choose from {sorted(mixed_precision_policies)})") from None


if __name__ == "__main__":
    for k, v in mixed_precision_policies.items():
        print(f"{k:12s} {v}")
