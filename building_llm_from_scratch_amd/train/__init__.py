from .optim import FusedAdamW, OptSlot, local_slots  # noqa: F401
