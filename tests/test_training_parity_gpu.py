"""Training over 50 steps: the GPU bf16 kernel path tracks the CPU fp32 path step by step.

Two tiny models, each trained 50 optimizer steps (AdamW, wd 0.1, clip 1.0) on the same cycle of
batches from the same initial weights:
* Llama (GQA, hd 64) with ``full`` activation checkpointing (every block recomputed);
* GPT-2 with dropout 0.1 (attention, residual and embedding dropout: the counter-hash masks are
  a function of (seed, element offset), so the CPU oracle drops the same elements).

Band.  A bf16 run differs from fp32 by rounding errors of relative size u = 2^-8 in every
operation, and training amplifies early differences.  The band is derived from the rounding unit
by measuring that amplification on the CPU: a second fp32 run whose initial weights are rounded
to bf16 (a perturbation of at most u per weight) gives the gap d_k that ONE u-sized
perturbation grows into by step k.  The bf16 path perturbs every step, so its gap may be a few
times larger than d_k; on top of that each step's loss is a mean over n = 512 token losses whose
bf16 rounding errors (relative u each) are independent, so they leave about u L / sqrt(n) in the
mean:  |L_gpu(k) - L_cpu(k)| <= 8 d_k + 4 u L_cpu(k) / sqrt(n).  (Calibration on MI355X: the
largest gap was 0.03 of the looser band 8 d_k + 4 u L_cpu(k), i.e. about 0.7 of this one's
second term alone.)  The per-step gaps, d_k and the band are written to
gpurun_out/training_parity_<model>.json when that directory exists (profiles/r4/ keeps a copy)."""
import json
import os

import pytest
import torch

from building_llm_from_scratch_amd import ops
from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.models import build_model
from building_llm_from_scratch_amd.train.optim import FusedAdamW

pytestmark = pytest.mark.gpu

U_BF16 = 2.0 ** -8
STEPS = 50


def _cfg(name):
    if name == "llama_full_ckpt":
        return get_config("llama3_2", "1B").replace(context_length=128, emb_dim=256, n_heads=4, n_kv_groups=2,
                                                    hidden_dim=512, n_layers=2, vocab_size=512), "full"
    return get_config("GPT2", "124M").replace(context_length=128, emb_dim=256, n_heads=4, n_kv_groups=4,
                                              hidden_dim=1024, n_layers=2, vocab_size=512, drop_rate=0.1), "none"


def _run(model, batches, device):
    opt = FusedAdamW(model, lr=1e-3, weight_decay=0.1)
    model.train()
    losses = []
    for k in range(STEPS):
        b = batches[k % len(batches)].to(device)
        opt.zero_grad()
        loss = model(b[:, :-1], b[:, 1:])
        loss.backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        losses.append(float(loss.item()))
    return losses


@pytest.mark.parametrize("name", ["llama_full_ckpt", "gpt2_dropout"])
def test_50_step_bf16_loss_curve_tracks_cpu_fp32(name):
    ops.load_ext(required=True)
    cfg, ckpt = _cfg(name)
    g = torch.Generator().manual_seed(3)
    batches = [torch.randint(0, cfg.vocab_size, (4, 129), generator=g) for _ in range(6)]
    torch.manual_seed(0)
    ref = build_model(cfg.replace(dtype=torch.float32), use_actv_ckpt=ckpt)
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    cpu = _run(ref, batches, "cpu")
    # the same fp32 run from bf16-rounded initial weights: how a u-sized perturbation grows
    pert = build_model(cfg.replace(dtype=torch.float32), use_actv_ckpt=ckpt)
    pert.load_state_dict({k: v.to(torch.bfloat16).float() for k, v in init.items()})
    cpu_p = _run(pert, batches, "cpu")
    gpu_m = build_model(cfg.replace(dtype=torch.bfloat16), use_actv_ckpt=ckpt, device="cuda")
    gpu_m.load_state_dict(init)
    gpu = _run(gpu_m, batches, "cuda")
    d = [abs(a - b) for a, b in zip(cpu, cpu_p)]
    n_tok = batches[0].shape[0] * (batches[0].shape[1] - 1)
    band = [8 * dk + 4 * U_BF16 * abs(lk) / n_tok ** 0.5 for dk, lk in zip(d, cpu)]
    gap = [abs(a - b) for a, b in zip(gpu, cpu)]
    rec = {"model": name, "ckpt": ckpt, "steps": STEPS, "u_bf16": U_BF16, "loss_cpu_fp32": cpu,
           "loss_gpu_bf16": gpu, "gap": gap, "d_u_perturbation": d, "band": band,
           "max_gap_over_band": max(x / y for x, y in zip(gap, band))}
    if os.path.isdir("gpurun_out"):
        with open(os.path.join("gpurun_out", f"training_parity_{name}.json"), "w") as f:
            json.dump(rec, f, indent=1)
    assert cpu[-1] < cpu[0] - 1.0, cpu                 # the run really trains
    bad = [(k, gap[k], band[k]) for k in range(STEPS) if gap[k] > band[k]]
    assert not bad, bad[:5]
