#!/usr/bin/env python3
"""Reference-compatible entry point: ``python main.py [flags]`` (reference main.py:185-193).
See ``python main.py --help`` and building_llm_from_scratch_amd/cli.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from building_llm_from_scratch_amd.cli import cli  # noqa: E402

if __name__ == "__main__":
    cli()
