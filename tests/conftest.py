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


@pytest.fixture(scope="session")
def ctx_dict():
    """A context that builds the wc hot-key dictionary even for small splits
    (default: only splits >= 32 MiB get one), so parity covers the dictionary path."""
    from mrgpu import Context

    c = Context(0)
    c.set_option("dict_min_bytes", 1)
    yield c
    c.close()


@pytest.fixture(params=["nodict", "dict"])
def wctx(request):
    """wc parity runs on both paths: no dictionary (every word spills) and dictionary."""
    return request.getfixturevalue("ctx" if request.param == "nodict" else "ctx_dict")
