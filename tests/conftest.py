import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running physics test")
    # build the in-tree native core if it is missing (hipcc cross-compiles for gfx950 on CPU hosts)
    import importlib.util

    so_present = any(f.startswith("_C") and f.endswith(".so") for f in os.listdir(os.path.join(ROOT, "channel_gpu_amd")))
    if not so_present:
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build.py"), "--no-driver"], check=True)


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    from channel_gpu_amd import require_native

    return require_native()
