import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-systems-implemented_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X; runs the HIP library through the C ABI")


@pytest.fixture(scope="session")
def ctx():
    """One GPU context for the whole gpu-marked session (fails loudly without a GPU)."""
    from mrgpu import Context

    c = Context(0)
    yield c
    c.close()
