import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


_HB_STREAM = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # pytest's fd-level capture redirects fd 2 (sys.__stderr__ included) while a test runs:
    # the heartbeat writes to a duplicate of the fd 2 pytest saved before capturing
    global _HB_STREAM
    try:
        capman = config.pluginmanager.getplugin("capturemanager")
        fd = capman._global_capturing.err.targetfd_save
        _HB_STREAM = os.fdopen(os.dup(fd), "w")
    except Exception:
        _HB_STREAM = None


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


@pytest.fixture(autouse=True)
def _heartbeat(request):
    """A line on stderr every 60 s while a test runs: the GPU box's runner takes a run that
    writes nothing for 3 minutes to be hung, and some oracle evaluations (fp64 CPU passes of
    a whole training step at 512x1024) take longer than that."""
    import threading
    import time
    stop = threading.Event()
    t0 = time.time()

    def beat():
        while not stop.wait(60):
            print(f"[heartbeat] {request.node.nodeid} running {time.time() - t0:.0f}s",
                  file=_HB_STREAM or sys.__stderr__, flush=True)

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
    th.join(timeout=5)
