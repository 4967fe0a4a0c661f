import os
import sys

import pytest
# torch first: it bundles its own libamdhip64 (same SONAME as /opt/rocm's,
# which libaclswarm_amd.so links). Loaded first, torch's copy is the one HIP
# runtime of the process and the in-tree libraries bind to it; a test that
# ctypes-loads a driver library before torch would instead bring in
# /opt/rocm's runtime, and torch then finds no device ("No HIP GPUs are
# available", seen when tests/test_gpu_facade.py ran before any torch test).
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
