import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _test_local_env():
    """Environment knobs a test (or a helper it calls) sets -- DVIE_PRECISION, the
    DVIE_* kernel overrides -- are restored after it, so no test inherits another's
    precision or kernel choice whatever the order they run in."""
    saved = {k: v for k, v in os.environ.items() if k.startswith("DVIE_")}
    yield
    for k in [k for k in os.environ if k.startswith("DVIE_")]:
        if k not in saved:
            del os.environ[k]
    os.environ.update(saved)
