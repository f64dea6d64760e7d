"""The native C++ BPE core (csrc/host/bpe.cpp) must reproduce the pure-Python regex +
merge path exactly, for the GPT-2 and the Llama-3 pre-tokenisation patterns."""
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from building_llm_from_scratch_amd.data.tokenizer import GPT2_PAT, LLAMA3_PAT, BPETokenizer

_bpe = pytest.importorskip("building_llm_from_scratch_amd._bpe")

RANKS = {bytes([i]): i for i in range(256)}
for w in ["th", "he", "in", "the", "an", "er", "on", " the", " a", "'s", "re", "ll", "12", "123", "\n\n",
          "  ", "ü", " w", "wo", "wor", "word"]:
    RANKS.setdefault(w.encode(), len(RANKS))

ALPHABET = st.sampled_from(list("aAbeélnorstTwWü中文 \t\n\r'’—“”.,!?-0123456789٣  ") + ["'s", "'RE", "'ll"])


@pytest.mark.parametrize("pat", [GPT2_PAT, LLAMA3_PAT], ids=["gpt2", "llama3"])
@settings(max_examples=300, deadline=None)
@given(parts=st.lists(ALPHABET, max_size=60))
def test_native_matches_python(pat, parts):
    text = "".join(parts)
    tok = BPETokenizer(RANKS, pat)
    assert tok._native_core() is not None
    assert tok.encode_ordinary(text) == tok._encode_ordinary_py(text)


@pytest.mark.parametrize("pat", [GPT2_PAT, LLAMA3_PAT], ids=["gpt2", "llama3"])
def test_native_matches_python_book(pat):
    import random
    from building_llm_from_scratch_amd.data.synthetic import _lexicon, synthetic_book
    rng = random.Random(1)
    text = synthetic_book(rng, _lexicon(rng, 500), 3000) + " It’s 2024 — “quoted”\r\n\n  x\t\ty  "
    tok = BPETokenizer(RANKS, pat)
    assert tok.encode_ordinary(text) == tok._encode_ordinary_py(text)
    assert tok.decode(tok.encode_ordinary(text)) == text
