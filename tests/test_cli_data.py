"""CPU tests: CLI surface + validation (reference args.py), datasets / collate masking
(datautils/*), dataset prep, tokenizers, mixed-precision policies, LR schedule, sampling and
the checkpoint layout."""
import json
import math
import os

import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from building_llm_from_scratch_amd import cli
from building_llm_from_scratch_amd.config import get_config
from building_llm_from_scratch_amd.data import ByteTokenizer, DatasetPT, custom_collate_fn
from building_llm_from_scratch_amd.data.prepare import combine_files, is_english, load_alpaca, strip_headers
from building_llm_from_scratch_amd.data.tokenizer import BPETokenizer, _bytes_to_unicode
from building_llm_from_scratch_amd.models import build_model, replace_linear_with_lora
from building_llm_from_scratch_amd.parallel.mixed_precision import (bf16_hybrid_policy, bf16_policy, fp16_policy,
                                                                    fp32_policy, get_policy, mixed_precision_policies)
from building_llm_from_scratch_amd.train.checkpoint import load_model, save_model
from building_llm_from_scratch_amd.train.generate import generate
from building_llm_from_scratch_amd.train.trainer import Trainer

REFERENCE_FLAGS = {  # args.py:46-93 — name: default
    "data_dir": "/home/ec2-user/train-llm-from-scratch/Datasets/Gutenberg/data_dir_small",
    "output_dir": "model_checkpoints", "n_epochs": 2, "batch_size": 4, "lr": 5e-4, "warmup_steps": 10,
    "initial_lr": 1e-5, "min_lr": 1e-6, "print_sample_iter": 10, "eval_freq": 10, "save_ckpt_freq": 100,
    "model": "GPT2", "num_params": "124M", "load_weights": False, "debug": False, "run_type": "single_gpu",
    "use_fsdp": False, "use_zero_opt": False, "use_actv_ckpt": False, "data_type": "fp32",
    "mixed_precision": None, "finetune": False, "dataset": "gutenberg", "use_lora": False, "lora_rank": 64,
    "lora_alpha": 32, "warnings": False,
}


# ---------------------------------------------------------------------------- CLI
def test_reference_flags_and_defaults():
    ns = cli.build_parser().parse_args([])
    for k, v in REFERENCE_FLAGS.items():
        assert getattr(ns, k) == v, k
    assert len(REFERENCE_FLAGS) == 27


@pytest.mark.parametrize("extra,err", [
    (["--model", "GPT2", "--num_params", "8B"], ValueError),
    (["--use_fsdp"], ValueError),                                        # FSDP needs multi_gpu
    (["--run_type", "multi_gpu", "--use_fsdp", "--use_zero_opt"], ValueError),
    (["--mixed_precision", "bf16"], ValueError),                         # needs FSDP
    # the auto planner picks the recomputed blocks; a segment count would silently replace it
    (["--use_actv_ckpt", "--actv_ckpt_mode", "auto", "--actv_ckpt_segments", "4"], ValueError),
])
def test_perform_checks_rejects(tmp_path, extra, err):
    with pytest.raises(err):
        cli.get_args(["--data_dir", str(tmp_path)] + extra)


def test_perform_checks_missing_dir(tmp_path):
    with pytest.raises(FileNotFoundError):
        cli.get_args(["--data_dir", str(tmp_path / "nope")])
    a = cli.get_args(["--data_dir", str(tmp_path / "made"), "--synthetic_data"])
    assert os.path.isdir(a.data_dir)


def test_perform_checks_accepts_valid(tmp_path):
    a = cli.get_args(["--data_dir", str(tmp_path), "--model", "llama3_2", "--num_params", "1B",
                      "--run_type", "multi_gpu", "--use_fsdp", "--mixed_precision", "bf16", "--backend", "gloo"])
    assert a.use_fsdp and a.mixed_precision == "bf16"


# ---------------------------------------------------------------------------- data
@settings(max_examples=40, deadline=None)
@given(n=st.integers(0, 300), L=st.integers(1, 40), stride=st.integers(1, 40))
def test_dataset_windows(n, L, stride):
    ids = torch.arange(n, dtype=torch.int32)
    ds = DatasetPT("", None, L, stride, token_ids=ids)
    assert len(ds) == len(range(0, n - L, stride))  # reference dataset.py:29
    for i in range(min(len(ds), 3)):
        x, y = ds[i]
        assert x.tolist() == list(range(i * stride, i * stride + L))
        assert y.tolist() == list(range(i * stride + 1, i * stride + L + 1))


def _collate_oracle(batch, pad, ignore, maxlen):
    """Independent restatement of dataloader_instruction_finetune.py:20-50."""
    longest = max(len(t) for _, t in batch) + 1
    xs, ys = [], []
    for ilen, toks in batch:
        seq = list(toks) + [pad] * (longest - len(toks))
        x, y = seq[:-1], seq[1:]
        first_pad_seen = False
        for j, v in enumerate(y):
            if v == pad:
                if first_pad_seen:
                    y[j] = ignore
                first_pad_seen = True
        for j in range(min(max(ilen - 1, 0), len(y))):
            y[j] = ignore
        if maxlen is not None:
            x, y = x[:maxlen], y[:maxlen]
        xs.append(x)
        ys.append(y)
    return xs, ys


@settings(max_examples=60, deadline=None)
@given(items=st.lists(st.tuples(st.integers(0, 6), st.lists(st.integers(0, 20), min_size=1, max_size=12)),
                      min_size=1, max_size=4),
       maxlen=st.one_of(st.none(), st.integers(1, 10)))
def test_collate_masking(items, maxlen):
    pad = 7
    x, y = custom_collate_fn(items, pad_token_id=pad, allowed_max_length=maxlen)
    ox, oy = _collate_oracle(items, pad, -100, maxlen)
    assert x.tolist() == ox and y.tolist() == oy


def test_collate_survey_example():
    # targets [-100, 9, 50256, -100, -100]
    x, y = custom_collate_fn([(2, [5, 8, 9]), (1, [1, 2, 3, 4, 6])])
    assert y[0].tolist() == [-100, 9, 50256, -100, -100]
    assert x[0].tolist() == [5, 8, 9, 50256, 50256]


def test_phi_format_dataset():
    """Phi-format formatter and dataset (reference dataset_instruction_finetune.py:28-99); items
    carry the prompt length so the reference collate masks the prompt."""
    from building_llm_from_scratch_amd.data.datasets import InstructionDatasetPhi, format_input_phi
    e1 = {"instruction": "Add.", "input": "1 2", "output": "3"}
    e2 = {"instruction": "Greet.", "input": "", "output": "hi"}
    assert format_input_phi(e1) == "<|user|>\nAdd.\n1 2"
    assert format_input_phi(e2) == "<|user|>\nGreet."
    tok = ByteTokenizer()
    ds = InstructionDatasetPhi([e1, e2], tok)
    n, ids = ds[0]
    assert tok.decode(ids) == "<|user|>\nAdd.\n1 2\n<|assistant|>:\n3"
    assert n == len(tok.encode(format_input_phi(e1))) and len(ds) == 2
    x, y = custom_collate_fn([ds[0], ds[1]], pad_token_id=0)
    assert (y[0, :n - 1] == -100).all() and y[0, n - 1] != -100


# ---------------------------------------------------------------------------- prep
def test_prepare_gutenberg(tmp_path):
    src = tmp_path / "txt"
    (src / "sub").mkdir(parents=True)
    hdr = "Title\n*** START OF THE PROJECT GUTENBERG EBOOK X ***\n"
    ftr = "\n*** END OF THE PROJECT GUTENBERG EBOOK X ***\nlicence text"
    (src / "a.txt").write_text(hdr + "Body one.\n\n\n\nMore." + ftr)
    (src / "sub" / "b.txt").write_text(hdr + "Body two." + ftr)
    (src / "c.txt").write_text("ЖЖЖЖЖЖЖЖЖЖ non english ЖЖЖЖЖЖЖЖЖЖЖЖЖ")
    from building_llm_from_scratch_amd.data.prepare import find_text_files
    files = find_text_files(str(src))
    assert len(files) == 3
    n = combine_files(files, str(tmp_path / "out"), max_size_mb=1)
    assert n == 1
    out = (tmp_path / "out" / "combined_1.txt").read_text()
    assert out == "Body one.\n\nMore.<|endoftext|>Body two."
    # size limit -> one book per file
    n = combine_files([files[0], files[2]], str(tmp_path / "out2"), max_size_mb=1e-5)
    assert n == 2
    assert not is_english("ЖЖЖЖ a") and is_english("plain ascii")
    assert strip_headers("no markers") == "no markers"


def test_prepare_alpaca(tmp_path):
    recs = load_alpaca(str(tmp_path / "d" / "alpaca.json"), n_synthetic=20)
    assert len(recs) == 20 and set(recs[0]) >= {"instruction", "input", "output"}
    again = load_alpaca(str(tmp_path / "copy.json"), source=str(tmp_path / "d" / "alpaca.json"))
    assert again == recs


# ---------------------------------------------------------------------------- tokenizers
@settings(max_examples=50, deadline=None)
@given(text=st.text(max_size=60))
def test_byte_tokenizer_roundtrip(text):
    tok = ByteTokenizer({"<|endoftext|>": 50256})
    ids = tok.encode(text + "<|endoftext|>", allowed_special={"<|endoftext|>"})
    assert ids[-1] == 50256
    assert tok.decode(ids) == text + "<|endoftext|>"


def test_bpe_from_gpt2_files(tmp_path):
    b2u = _bytes_to_unicode()
    enc = {b2u[b]: i for i, b in enumerate(range(256))}
    merges = [("h", "e"), ("l", "l"), ("he", "ll"), ("hell", "o"), ("Ġ", "w")]
    for a, b in merges:
        enc[a + b] = len(enc)
    enc["<|endoftext|>"] = 50256
    (tmp_path / "encoder.json").write_text(json.dumps(enc))
    tok = BPETokenizer.from_gpt2_files(str(tmp_path / "encoder.json"))
    ids = tok.encode("hello world<|endoftext|>", allowed_special={"<|endoftext|>"})
    assert ids[0] == enc["hello"] and ids[1] == enc["Ġw"] and ids[-1] == 50256
    assert tok.decode(ids) == "hello world<|endoftext|>"


# ---------------------------------------------------------------------------- policies
def test_mixed_precision_policies():
    assert set(mixed_precision_policies) == {"fp16", "bf16", "bf16_hybrid", "fp32"}
    assert bf16_policy.param_dtype == torch.bfloat16 and bf16_policy.reduce_dtype == torch.bfloat16
    assert bf16_hybrid_policy.param_dtype == torch.float32 and bf16_hybrid_policy.reduce_dtype == torch.bfloat16
    assert fp16_policy.loss_scaling and not bf16_policy.loss_scaling and not fp32_policy.loss_scaling
    assert get_policy("bf16") is bf16_policy
    with pytest.raises(ValueError):
        get_policy("int8")


# ---------------------------------------------------------------------------- schedule
class _Opt:
    def __init__(self, lr):
        self.param_groups = [{"lr": lr}]


class _Loader:
    def get_total_steps_epoch(self, files):
        return 50


def test_lr_schedule_matches_reference_formula():
    tr = Trainer(model=None, optimizer=_Opt(5e-4), config={}, data_files=["a"], loaderObj=_Loader(),
                 save_dir="/tmp/none", warmup_steps=10, initial_lr=1e-5, min_lr=1e-6)
    tr._setup_schedule(n_epochs=2)
    total, inc = 100, (5e-4 - 1e-5) / 10
    for step in (0, 5, 9, 10, 40, 99):
        if step < 10:
            ref = 1e-5 + step * inc
        else:
            ref = 1e-6 + (5e-4 - 1e-6) * 0.5 * (1 + math.cos(math.pi * (step - 10) / (total - 10)))
        assert abs(tr.lr_at(step) - ref) < 1e-12, step


# ---------------------------------------------------------------------------- checkpoint layout
def _cfg(model, size, **kw):
    from building_llm_from_scratch_amd.config import debug_config
    return debug_config(get_config(model, size)).replace(dtype=torch.float32, **kw)


def test_gpt2_state_dict_layout():
    cfg = _cfg("GPT2", "124M", qkv_bias=True)
    sd = build_model(cfg).state_dict()
    T, d, V = cfg.context_length, cfg.emb_dim, cfg.vocab_size
    assert sd["tok_emb.weight"].shape == (V, d) and sd["pos_emb.weight"].shape == (T, d)
    for i in range(cfg.n_layers):
        p = f"blocks.{i}."
        assert sd[p + "att.mask"].shape == (T, T)
        for n in ("W_query", "W_key", "W_value", "out_proj"):
            assert sd[p + f"att.{n}.weight"].shape == (d, d) and sd[p + f"att.{n}.bias"].shape == (d,)
        assert sd[p + "ff.layers.0.weight"].shape == (4 * d, d) and sd[p + "ff.layers.2.weight"].shape == (d, 4 * d)
        for n in ("norm1", "norm2"):
            assert sd[p + f"{n}.weight"].shape == (d,) and sd[p + f"{n}.bias"].shape == (d,)
    assert sd["norm.weight"].shape == (d,) and sd["output_head.weight"].shape == (V, d)
    assert all(v.dtype == torch.float32 for v in sd.values())
    n_expected = 2 + cfg.n_layers * (1 + 8 + 4 + 4) + 3
    assert len(sd) == n_expected


@pytest.mark.parametrize("model,size", [("llama3", "8B"), ("llama2", "7B"), ("llama3_2", "1B")])
def test_llama_state_dict_layout(model, size):
    cfg = _cfg(model, size).replace(dtype=torch.bfloat16)
    sd = build_model(cfg).state_dict()
    T, d, V, F = cfg.context_length, cfg.emb_dim, cfg.vocab_size, cfg.hidden_dim
    hd, G = d // cfg.n_heads, cfg.n_kv_groups
    assert sd["tok_emb.weight"].shape == (V, d) and sd["tok_emb.weight"].dtype == torch.bfloat16
    for i in range(cfg.n_layers):
        p = f"trf_blocks.{i}."
        assert sd[p + "att.mask"].shape == (T, T)
        assert sd[p + "att.cos"].shape == (T, hd) and sd[p + "att.sin"].shape == (T, hd)
        assert sd[p + "att.W_query.weight"].shape == (d, d)
        assert sd[p + "att.W_key.weight"].shape == (G * hd, d) and sd[p + "att.W_value.weight"].shape == (G * hd, d)
        assert sd[p + "ff.fc1.weight"].shape == (F, d) and sd[p + "ff.fc3.weight"].shape == (d, F)
        assert sd[p + "norm1.weight"].dtype == torch.float32
    assert sd["final_norm.weight"].dtype == torch.float32 and sd["out_head.weight"].shape == (V, d)
    cos_dt = torch.float32 if model == "llama2" else torch.bfloat16
    assert sd["trf_blocks.0.att.cos"].dtype == cos_dt


def test_lora_state_dict_layout():
    cfg = _cfg("llama3_2", "1B")
    m = build_model(cfg)
    for p in m.parameters():
        p.requires_grad = False
    replace_linear_with_lora(m, rank=4, alpha=8)
    sd = m.state_dict()
    d = cfg.emb_dim
    assert sd["trf_blocks.0.att.W_query.linear.weight"].shape == (d, d)
    assert sd["trf_blocks.0.att.W_query.lora.A"].shape == (d, 4)
    assert sd["trf_blocks.0.att.W_query.lora.B"].shape == (4, d)
    assert "out_head.lora.A" in sd and "out_head.linear.weight" in sd


def test_checkpoint_roundtrip(tmp_path):
    cfg = _cfg("GPT2", "124M")
    torch.manual_seed(0)
    a = build_model(cfg)
    torch.manual_seed(1)
    b = build_model(cfg)
    save_model(a, tmp_path / "model_pg_0.pth")
    load_model(b, tmp_path / "model_pg_0.pth")
    sa, sb = a.state_dict(), b.state_dict()
    assert all(torch.equal(sa[k], sb[k]) for k in sa)
    raw = torch.load(tmp_path / "model_pg_0.pth", weights_only=True)
    assert list(raw) == list(sa)  # plain, prefix-free, same order


# ---------------------------------------------------------------------------- sampling
def test_generate_greedy_matches_manual_loop():
    cfg = _cfg("llama3_2", "1B")
    torch.manual_seed(0)
    m = build_model(cfg)
    m.flatten()
    idx = torch.randint(0, cfg.vocab_size, (2, 4))
    out = generate(m, idx, max_new_tokens=5, context_size=cfg.context_length)
    cur = idx.clone()
    with torch.no_grad():
        for _ in range(5):
            logits = m(cur[:, -cfg.context_length:])[:, -1, :]
            cur = torch.cat([cur, logits.argmax(-1, keepdim=True)], 1)
    assert torch.equal(out, cur)


@pytest.mark.parametrize("model,size,G", [("llama3_2", "1B", 2), ("GPT2", "124M", 4), ("llama2", "7B", 4)])
def test_generate_cached_matches_recompute(model, size, G):
    """KV-cache decode (incl. the sliding-window re-prefill) == the reference's full recompute."""
    from building_llm_from_scratch_amd.train.generate import generate_cached
    cfg = get_config(model, size).replace(context_length=24, emb_dim=64, n_heads=4, n_kv_groups=G, hidden_dim=96,
                                          n_layers=2, vocab_size=101, dtype=torch.float32, drop_rate=0.0)
    torch.manual_seed(0)
    m = build_model(cfg)
    m.flatten()
    idx = torch.randint(0, 101, (2, 5))
    assert torch.equal(generate(m, idx, 30, 24), generate_cached(m, idx, 30, 24))
    g1, g2 = torch.Generator().manual_seed(3), torch.Generator().manual_seed(3)
    a = generate(m, idx, 12, 24, temperature=1.0, top_k=5, generator=g1)
    b = generate_cached(m, idx, 12, 24, temperature=1.0, top_k=5, generator=g2)
    assert torch.equal(a, b)


@pytest.mark.parametrize("check_every", [1, 4, 16])
@pytest.mark.parametrize("rows", [1, 2])
def test_generate_cached_eos_stop_matches_reference(check_every, rows, monkeypatch):
    """Deferred all-rows-eos test (every ``EOS_CHECK_EVERY`` tokens) cuts the output exactly
    where the reference's per-token check stops (generate.py:68-70), for eos hits early, late,
    at a check boundary and never."""
    from building_llm_from_scratch_amd.train import generate as G
    monkeypatch.setattr(G, "EOS_CHECK_EVERY", check_every)
    cfg = get_config("llama3_2", "1B").replace(context_length=24, emb_dim=64, n_heads=4, n_kv_groups=2,
                                              hidden_dim=96, n_layers=2, vocab_size=7, dtype=torch.float32)
    torch.manual_seed(1)
    m = build_model(cfg)
    m.flatten()
    idx = torch.randint(0, 7, (rows, 3))
    free = G.generate(m, idx, 40, 24)                  # greedy, no eos: a short-vocab sequence
    for eos in range(7):
        ref = G.generate(m, idx, 40, 24, eos_id=eos)
        got = G.generate_cached(m, idx, 40, 24, eos_id=eos)
        assert torch.equal(ref, got), (eos, ref.shape, got.shape)
    assert free.shape[1] == 43


def test_multi_gpu_loaders_use_shuffling_distributed_sampler():
    """Under multi_gpu both loaders take DistributedSampler(dataset) with its default shuffle,
    as the reference (datautils/dataloader.py:50, dataloader_instruction_finetune.py:94): the
    validation batches that calc_loss_loader evaluates come from a seeded random subset."""
    import torch.distributed as dist
    from torch.utils.data.distributed import DistributedSampler

    from building_llm_from_scratch_amd.data.loaders import DataloaderIF, DataloaderPT
    from building_llm_from_scratch_amd.data.tokenizer import ByteTokenizer
    port = _free_port()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        tok = ByteTokenizer({"<|endoftext|>": 256})
        pt = DataloaderPT(tok, batch_size=2, max_length=8, stride=8, run_type="multi_gpu", cache_dir=None)
        train, val = pt.create_dataloaders("hello world, " * 200)
        recs = [{"instruction": f"say {i}", "input": "", "output": f"{i}"} for i in range(50)]
        tr2, va2 = DataloaderIF(tok, batch_size=2, max_length=64, run_type="multi_gpu").create_dataloaders(recs)
        for dl in (train, val, tr2, va2):
            assert isinstance(dl.sampler, DistributedSampler) and dl.sampler.shuffle
    finally:
        dist.destroy_process_group()


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("multi", [False, True])
def test_first_batches_match_worker_loader(multi):
    """Evaluation reads its eval_iter batches through data.loaders.first_batches: the same
    batches iter(loader) yields, without forking the loader's worker processes."""
    from building_llm_from_scratch_amd.data.loaders import DataloaderIF, DataloaderPT, first_batches
    from building_llm_from_scratch_amd.data.tokenizer import ByteTokenizer
    import torch.distributed as dist
    if multi:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        tok = ByteTokenizer({"<|endoftext|>": 256})
        rt = "multi_gpu" if multi else "single_gpu"
        pt = DataloaderPT(tok, batch_size=3, max_length=8, stride=8, run_type=rt, cache_dir=None)
        recs = [{"instruction": f"say {i}", "input": "", "output": f"{i}" * (i % 7)} for i in range(40)]
        collate = __import__("functools").partial(custom_collate_fn, pad_token_id=256, allowed_max_length=64)
        dif = DataloaderIF(tok, batch_size=2, max_length=64, run_type=rt, collate_func=collate)
        for mk in (lambda w: pt.create_dataloaders("hello world, " * 200, num_workers=w)[1],
                   lambda w: dif.create_dataloaders(recs, num_workers=w)[1]):
            ref = [b for _, b in zip(range(4), mk(0))]
            got = list(first_batches(mk(2), 4))
            assert len(got) == len(ref) >= 2
            for (a, b), (c, d) in zip(got, ref):
                assert torch.equal(a, c) and torch.equal(b, d)
        assert list(first_batches(mk(2), 0)) == []
    finally:
        if multi:
            dist.destroy_process_group()


def test_tunableop_table_resolution(tmp_path, monkeypatch):
    """--tunableop auto picks the shipped MI355X table of the model / size; a copy (never the
    shipped file) is what TunableOp is pointed at, read-only."""
    from building_llm_from_scratch_amd.utils import gemm_tuning as gt
    assert gt.resolve_table("auto", "llama3", "8B").endswith("tunableop_llama3_8b_b40_mi355x.csv")
    assert gt.resolve_table("auto", "GPT2", "774M").endswith("tunableop_gpt2_774m_b64_mi355x.csv")
    assert gt.resolve_table("auto", "llama3_2", "1B") is None
    assert gt.resolve_table("none", "llama3", "8B") is None and gt.resolve_table(None) is None
    with pytest.warns(UserWarning, match="not found"):
        assert gt.resolve_table(str(tmp_path / "missing.csv")) is None
    for k in ("PYTORCH_TUNABLEOP_ENABLED", "PYTORCH_TUNABLEOP_TUNING", "PYTORCH_TUNABLEOP_FILENAME"):
        monkeypatch.delenv(k, raising=False)
    assert gt.install_table(None) is None and "PYTORCH_TUNABLEOP_ENABLED" not in os.environ
    src = gt.resolve_table("configs/tunableop_gpt2_774m_b64_mi355x.csv")
    d = gt.install_table(src, local_rank=3)
    assert os.environ["PYTORCH_TUNABLEOP_TUNING"] == "0"
    cp = os.environ["PYTORCH_TUNABLEOP_FILENAME"].replace("%d", "3")
    assert os.path.dirname(cp) == d and open(cp).read() == open(src).read()
    assert not os.path.islink(cp)
    assert cli.build_parser().parse_args([]).tunableop == "auto"


def test_trainer_reuses_loaders_across_epochs(tmp_path):
    """With few data files the trainer builds a file's loaders once and, each later epoch,
    reseeds their shuffle generator (persistent workers are forked once): every epoch sees the
    batch order that fresh loaders seeded for that (epoch, file) give."""
    import json
    from building_llm_from_scratch_amd.data.loaders import DataloaderIF
    from building_llm_from_scratch_amd.data.tokenizer import ByteTokenizer
    from building_llm_from_scratch_amd.utils.misc import read_json_file
    tok = ByteTokenizer({"<|endoftext|>": 256})
    recs = [{"instruction": f"say {i}", "input": "", "output": f"{i}" * (1 + i % 5)} for i in range(40)]
    fp = tmp_path / "a.json"
    fp.write_text(json.dumps(recs))
    collate = __import__("functools").partial(custom_collate_fn, pad_token_id=256, allowed_max_length=256)
    dif = DataloaderIF(tok, batch_size=4, max_length=256, collate_func=collate)
    made = []
    orig = dif.create_dataloaders
    dif.create_dataloaders = lambda *a, **k: (made.append(1), orig(*a, **k))[1]
    tr = Trainer(model=None, optimizer=_Opt(5e-4), config={}, data_files=[str(fp)], loaderObj=dif,
                 save_dir=str(tmp_path), num_workers=2, seed=123)
    seen = []
    tr.train_epoch = lambda epoch, tl, vl, **kw: seen.append([x.clone() for x, _ in tl])
    tr._loop(3, read_json_file, "ctx")
    assert len(made) == 1 + 1        # get_total_steps_epoch's + the first epoch's; epochs 2-3 reuse
    for epoch, got in enumerate(seen):
        g = torch.Generator().manual_seed(123 * 1_000_003 + epoch * 1009)
        ref = [x for x, _ in orig(recs, num_workers=0, generator=g)[0]]
        assert len(got) == len(ref) == 9
        assert all(torch.equal(a, b) for a, b in zip(got, ref)), epoch
    assert not all(a.shape == b.shape and torch.equal(a, b) for a, b in zip(seen[0], seen[1]))   # reshuffled


def test_gemm_epilogues_flag(tmp_path, monkeypatch):
    """``--gemm_epilogues`` turns on the three fused forward epilogues (gate/up + SwiGLU, QKV +
    RoPE, c_fc + bias + GELU on csrc/gemm_nt.hip); off by default (measured slower, README)."""
    import torch
    from building_llm_from_scratch_amd.builder import build_model as build_model_
    from building_llm_from_scratch_amd.config import get_config
    from building_llm_from_scratch_amd.models import linear
    for k in ("FUSED_SWIGLU", "FUSED_ROPE", "FUSED_GELU"):
        monkeypatch.setattr(linear, k, False)
    cfg = get_config("llama3_2", "1B").replace(context_length=16, emb_dim=32, n_heads=2, n_kv_groups=1,
                                                hidden_dim=48, n_layers=1, vocab_size=97, dtype=torch.float32)
    a = cli.get_args(["--data_dir", str(tmp_path), "--model", "llama3_2", "--num_params", "1B", "--device", "cpu"])
    a.world_size = 1
    build_model_(cfg, 0, torch.device("cpu"), a)
    assert not (linear.FUSED_SWIGLU or linear.FUSED_ROPE or linear.FUSED_GELU)
    a = cli.get_args(["--data_dir", str(tmp_path), "--model", "llama3_2", "--num_params", "1B", "--device", "cpu",
                      "--gemm_epilogues"])
    a.world_size = 1
    build_model_(cfg, 0, torch.device("cpu"), a)
    assert linear.FUSED_SWIGLU and linear.FUSED_ROPE and linear.FUSED_GELU
