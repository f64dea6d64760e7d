"""Synthetic, offline stand-ins for the reference's dataset prep scripts.

* Gutenberg (reference Datasets/Gutenberg/prepare_dataset.py:14-61): books are cleaned,
  blank lines collapsed, and concatenated with ``<|endoftext|>`` into ``combined_N.txt``
  files of at most ``max_size_mb``.  :func:`make_gutenberg_corpus` writes files in exactly
  that format from a seeded Zipfian word model.
* Alpaca (reference Datasets/Alpaca/download.py:5-36): a JSON list of
  ``{"instruction", "input", "output"}`` records.  :func:`make_alpaca_json` writes the same
  shape (antonym / arithmetic / rewrite tasks so finetuning has learnable structure).
"""
from __future__ import annotations

import json
import os
import random
from typing import List

_SYLLABLES = ["ka", "lo", "mi", "ren", "tha", "vo", "sel", "dor", "an", "bri", "cu", "el",
              "fen", "gar", "hol", "is", "jun", "kel", "mor", "nes", "or", "pel", "qua", "ros",
              "sun", "tor", "ul", "ven", "wil", "yar", "zem", "the", "and", "ing", "ed", "er"]
_FUNCTION_WORDS = ["the", "of", "and", "to", "a", "in", "that", "he", "was", "it", "his",
                   "her", "with", "as", "had", "for", "she", "on", "at", "by", "not", "but"]


def _lexicon(rng: random.Random, n: int = 4000) -> List[str]:
    words = set(_FUNCTION_WORDS)
    while len(words) < n:
        k = rng.choice((1, 2, 2, 3, 3, 4))
        words.add("".join(rng.choice(_SYLLABLES) for _ in range(k)))
    lex = sorted(words)
    rng.shuffle(lex)
    return _FUNCTION_WORDS + [w for w in lex if w not in _FUNCTION_WORDS]


def synthetic_book(rng: random.Random, lexicon: List[str], n_words: int) -> str:
    weights = [1.0 / (i + 1) ** 1.07 for i in range(len(lexicon))]
    out, sent, para = [], [], []
    words = rng.choices(lexicon, weights=weights, k=n_words)
    for i, w in enumerate(words):
        sent.append(w)
        if len(sent) >= rng.randint(6, 22):
            s = " ".join(sent)
            para.append(s[0].upper() + s[1:] + rng.choice([".", ".", ".", "!", "?", ";"]))
            sent = []
            if len(para) >= rng.randint(3, 8):
                out.append(" ".join(para))
                para = []
    if sent:
        para.append(" ".join(sent) + ".")
    if para:
        out.append(" ".join(para))
    title = " ".join(w.capitalize() for w in rng.choices(lexicon[20:], k=3))
    return f"{title}\n\n" + "\n\n".join(out) + "\n"


def make_gutenberg_corpus(out_dir: str, n_files: int = 1, mb_per_file: float = 1.0,
                          seed: int = 123, separator: str = "<|endoftext|>") -> List[str]:
    """Write ``combined_1.txt`` ... ``combined_{n_files}.txt`` (books joined by ``separator``)."""
    os.makedirs(out_dir, exist_ok=True)
    rng = random.Random(seed)
    lex = _lexicon(rng)
    paths = []
    target = int(mb_per_file * 1024 * 1024)
    for fi in range(1, n_files + 1):
        books, size = [], 0
        while size < target:
            b = synthetic_book(rng, lex, rng.randint(2000, 8000))
            books.append(b)
            size += len(b) + len(separator)
        p = os.path.join(out_dir, f"combined_{fi}.txt")
        with open(p, "w", encoding="utf-8") as f:
            f.write(separator.join(books))
        paths.append(p)
    return paths


_ANTONYMS = [("hot", "cold"), ("big", "small"), ("fast", "slow"), ("happy", "sad"),
             ("complicated", "simple"), ("early", "late"), ("light", "dark"), ("rich", "poor"),
             ("strong", "weak"), ("open", "closed"), ("young", "old"), ("loud", "quiet")]


def make_alpaca_json(path: str, n_records: int = 1000, seed: int = 123) -> str:
    recs = alpaca_records(n_records, seed)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w", encoding="utf-8") as f:
        json.dump(recs, f, indent=1)
    return path


def alpaca_records(n_records: int = 1000, seed: int = 123) -> list:
    """Alpaca-shaped {instruction, input, output} records (reference Datasets/Alpaca/download.py
    fetches tatsu-lab's alpaca_data.json; no network here)."""
    rng = random.Random(seed)
    lex = _lexicon(rng, 800)
    recs = []
    for i in range(n_records):
        kind = i % 3
        if kind == 0:
            a, b = rng.choice(_ANTONYMS)
            recs.append({"instruction": f"What is an antonym of '{a}'?", "input": "",
                         "output": f"An antonym of '{a}' is '{b}'."})
        elif kind == 1:
            x, y = rng.randint(0, 99), rng.randint(0, 99)
            recs.append({"instruction": "Add the two numbers.", "input": f"{x} and {y}",
                         "output": f"The sum is {x + y}."})
        else:
            words = rng.choices(lex, k=rng.randint(4, 12))
            recs.append({"instruction": "Rewrite the sentence in reverse word order.",
                         "input": " ".join(words), "output": " ".join(reversed(words)) + "."})
    return recs


if __name__ == "__main__":  # python -m building_llm_from_scratch_amd.data.synthetic OUT_DIR
    import argparse
    ap = argparse.ArgumentParser(description="Write synthetic Gutenberg / Alpaca data")
    ap.add_argument("out_dir")
    ap.add_argument("--kind", choices=["gutenberg", "alpaca"], default="gutenberg")
    ap.add_argument("--n_files", type=int, default=1)
    ap.add_argument("--mb", type=float, default=1.0)
    ap.add_argument("--records", type=int, default=1000)
    a = ap.parse_args()
    if a.kind == "gutenberg":
        print(make_gutenberg_corpus(a.out_dir, a.n_files, a.mb))
    else:
        print(make_alpaca_json(os.path.join(a.out_dir, "instruction-data-alpaca.json"), a.records))
