"""Host-code AddressSanitizer/UBSan run of the native core's CPU components.

Builds csrc/core/{config,grid,plan,io}.cpp + tests/native/host_selftest.cpp with
-fsanitize=address,undefined (tools/host_sanitize.py) and requires a clean exit: malformed run.conf
inputs, every grid size, slab/pencil plans and UMEAN/HDF5 round trips without a sanitizer report.
CPU only."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(shutil.which("g++") is None and shutil.which("clang++") is None, reason="no host compiler")
def test_host_code_sanitizers_clean(tmp_path):
    import host_sanitize

    exe = host_sanitize.build(str(tmp_path))
    r = host_sanitize.run(exe)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
