import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
if os.environ.get("PYTEST_XDIST_WORKER"):
    # under pytest -n K every worker would otherwise run K x cpu_count intra-op threads next to
    # the gloo multi-process tests' ranks; the tiny CPU models gain nothing from more than two
    os.environ.setdefault("OMP_NUM_THREADS", "2")
    import torch
    torch.set_num_threads(int(os.environ["OMP_NUM_THREADS"]))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
