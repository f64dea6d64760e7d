"""the environment names the code reads are few (<= 15) and exactly the ones
README's "Environment knobs" table documents -- no undocumented A/B switch, no stale row."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["building_llm_from_scratch_amd", "csrc", "bench.py", "__graft_entry__.py", "main.py",
           os.path.join("tools", "build_ext.py")]
EXT = (".py", ".hip", ".h", ".cpp")


def _source_names():
    """Python: quoted BLLM_* names (os.environ reads) and NAME= forms (env dicts for child ranks,
    documented settings); C++: the names passed to getenv (the rest of BLLM_* there are macros)."""
    names = set()
    for entry in SOURCES:
        path = os.path.join(ROOT, entry)
        files = [path] if os.path.isfile(path) else [os.path.join(d, f) for d, _, fs in os.walk(path)
                                                     for f in fs if f.endswith(EXT)]
        for f in files:
            text = open(f, errors="replace").read()
            if f.endswith(".py"):
                names |= set(re.findall(r"[\"'](BLLM_[A-Z0-9_]+)[\"']", text))
                names |= set(re.findall(r"\b(BLLM_[A-Z0-9_]+)=", text))
            else:
                names |= set(re.findall(r"getenv\(\s*\"(BLLM_[A-Z0-9_]+)\"", text))
    return names


def _readme_names():
    text = open(os.path.join(ROOT, "README.md")).read()
    sec = text.split("## Environment knobs", 1)[1].split("\n## ", 1)[0]
    return set(re.findall(r"^\| `(BLLM_[A-Z0-9_]+)` \|", sec, flags=re.M))


def test_env_names_documented_and_few():
    src, doc = _source_names(), _readme_names()
    assert src == doc, {"undocumented": sorted(src - doc), "stale rows": sorted(doc - src)}
    assert len(src) <= 15, sorted(src)
