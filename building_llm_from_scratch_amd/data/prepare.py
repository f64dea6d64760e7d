"""Dataset preparation (reference ``Datasets/Gutenberg/prepare_dataset.py:9-89`` and
``Datasets/Alpaca/download.py:5-44``), offline.

Gutenberg: ``combine_files`` keeps predominantly-ASCII books, strips the Project Gutenberg
licence header/footer, collapses runs of blank lines and concatenates books with
``<|endoftext|>`` into ``combined_{n}.txt`` files of at most ``max_size_mb``.  The books are
streamed one at a time and each output file is written incrementally, so memory stays at one
book regardless of corpus size.  With no source directory (no network here) the synthetic
generator writes files of the same format (data/synthetic.py).

Alpaca: ``load_alpaca`` reads a local ``alpaca_data.json``-style file and writes it to the
path the instruction loader expects; without one it writes a synthetic file of the same shape.

CLI::

    python -m building_llm_from_scratch_amd.data.prepare gutenberg --data_dir txt/ --output_dir data_dir
    python -m building_llm_from_scratch_amd.data.prepare gutenberg --synthetic --output_dir data_dir
    python -m building_llm_from_scratch_amd.data.prepare alpaca --output data/instruction-data-alpaca.json
"""
from __future__ import annotations

import argparse
import json
import os
import re
from typing import Iterable, List, Optional

from .synthetic import make_alpaca_json, make_gutenberg_corpus

_BLANKS = re.compile(r"\n\s*\n")
# Project Gutenberg boilerplate markers (the header ends at the START line, the footer begins
# at the END line); older releases use "*END*THE SMALL PRINT" / "End of the Project Gutenberg".
_START = re.compile(r"^\s*\*{3}\s*START OF (THE|THIS) PROJECT GUTENBERG.*$|^\s*\*END\*THE SMALL PRINT.*$",
                    re.IGNORECASE | re.MULTILINE)
_END = re.compile(r"^\s*\*{3}\s*END OF (THE|THIS) PROJECT GUTENBERG.*$|^\s*End of (the )?Project Gutenberg.*$",
                  re.IGNORECASE | re.MULTILINE)


def is_english(text: str, threshold: float = 0.9) -> bool:
    """True when more than ``threshold`` of the characters are ASCII (reference :9-11)."""
    if not text:
        return False
    n_ascii = len(text.encode("ascii", "ignore"))
    return n_ascii / len(text) > threshold


def strip_headers(text: str) -> str:
    """Drop the Project Gutenberg licence header and footer, keep the book body."""
    start = 0
    m = None
    for m in _START.finditer(text):
        pass
    if m is not None:
        start = m.end()
    end = len(text)
    m2 = _END.search(text, start)
    if m2 is not None:
        end = m2.start()
    return text[start:end].strip("\n")


def _read(path: str, fallback_encoding: str = "latin1") -> str:
    try:
        with open(path, "r", encoding="utf-8") as f:
            return f.read()
    except UnicodeDecodeError:
        with open(path, "r", encoding=fallback_encoding) as f:
            return f.read()


def find_text_files(data_dir: str) -> List[str]:
    out = []
    for root, _, files in os.walk(data_dir):
        out.extend(os.path.join(root, n) for n in files if n.endswith(".txt"))
    return sorted(out)


def combine_files(file_paths: Iterable[str], target_dir: str, max_size_mb: float = 500,
                  separator: str = "<|endoftext|>", fallback_encoding: str = "latin1",
                  verbose: bool = False) -> int:
    """Returns the number of ``combined_{n}.txt`` files written."""
    os.makedirs(target_dir, exist_ok=True)
    limit = max_size_mb * 1024 * 1024
    counter, size, out = 1, 0, None
    n_in_file = 0

    def _open(n):
        return open(os.path.join(target_dir, f"combined_{n}.txt"), "w", encoding="utf-8")

    for path in file_paths:
        content = _read(path, fallback_encoding)
        if not is_english(content):
            if verbose:
                print(f"Skipping non-English file: {path}")
            continue
        content = _BLANKS.sub("\n\n", strip_headers(content))
        nbytes = len(content.encode("utf-8"))
        if out is not None and size + nbytes > limit and n_in_file > 0:
            out.close()
            counter += 1
            out, size, n_in_file = None, 0, 0
        if out is None:
            out = _open(counter)
        if n_in_file:
            out.write(separator)
        out.write(content)
        size += nbytes
        n_in_file += 1
    if out is None:
        return 0  # nothing kept
    out.close()
    return counter


def load_alpaca(output: str, source: Optional[str] = None, n_synthetic: int = 2000, seed: int = 123) -> list:
    """Write the Alpaca-format instruction file to ``output`` and return its records."""
    os.makedirs(os.path.dirname(os.path.abspath(output)), exist_ok=True)
    if source:
        with open(source, "r", encoding="utf-8") as f:
            data = json.load(f)
        with open(output, "w", encoding="utf-8") as f:
            json.dump(data, f, indent=1)
        return data
    make_alpaca_json(output, n_records=n_synthetic, seed=seed)
    with open(output, "r", encoding="utf-8") as f:
        return json.load(f)


def main(argv=None):
    ap = argparse.ArgumentParser(description="Offline dataset preparation")
    sub = ap.add_subparsers(dest="what", required=True)
    g = sub.add_parser("gutenberg")
    g.add_argument("--data_dir", default="Gutenberg/txt", help="directory of .txt books (recursive)")
    g.add_argument("--output_dir", default="data_dir")
    g.add_argument("--max_size_mb", type=float, default=500)
    g.add_argument("--synthetic", action="store_true", help="generate a synthetic corpus instead")
    g.add_argument("--synthetic_files", type=int, default=2)
    g.add_argument("--synthetic_mb", type=float, default=1.0)
    a = sub.add_parser("alpaca")
    a.add_argument("--output", default="data/instruction-data-alpaca.json")
    a.add_argument("--source", default=None, help="local alpaca_data.json (else synthetic)")
    a.add_argument("--n", type=int, default=2000)
    args = ap.parse_args(argv)
    if args.what == "gutenberg":
        if args.synthetic or not os.path.isdir(args.data_dir):
            paths = make_gutenberg_corpus(args.output_dir, n_files=args.synthetic_files, mb_per_file=args.synthetic_mb)
            print(f"{len(paths)} synthetic file(s) saved in: {os.path.abspath(args.output_dir)}")
        else:
            files = find_text_files(args.data_dir)
            print(f"Found {len(files)} text file(s) to process.")
            n = combine_files(files, args.output_dir, max_size_mb=args.max_size_mb, verbose=True)
            print(f"{n} file(s) saved in: {os.path.abspath(args.output_dir)}")
    else:
        data = load_alpaca(args.output, args.source, n_synthetic=args.n)
        print(f"Number of entries: {len(data)} -> {args.output}")


if __name__ == "__main__":
    main()
