import os
import sys

import pytest

# CPU threads per process: the multi-process tests run 2-8 ranks on this machine at once, each with torch's default
# of one OpenMP thread per CPU, i.e. up to 8x oversubscribed spin-waiting teams. A quarter of the CPUs per process
# unless the environment already says (the GPU boxes set OMP_NUM_THREADS); set before any test module imports torch,
# and inherited by the spawned ranks.
os.environ.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 8) // 4)))

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# SFTAMD_* variables present when the test session starts: the kernels read several of them per call, so a session
# started with overrides would not test the shipped default paths (tests/test_env_guard.py fails on any)
START_SFTAMD_ENV = {k: v for k, v in os.environ.items() if k.startswith("SFTAMD_")}


@pytest.fixture(autouse=True)
def _restore_environ():
    """Every test starts and ends with the session's environment: a test that sets a dispatch override (e.g. an
    attention variant) cannot leak it into the tests that run after it in the same process."""
    saved = dict(os.environ)
    yield
    if os.environ != saved:
        os.environ.clear()
        os.environ.update(saved)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
