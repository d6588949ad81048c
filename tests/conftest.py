import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "taiwan-whisper_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP library)")
    _heartbeat_start()


# a test that runs for minutes (the fp32 large-v2 long-form decode) prints a line every 60 s to the real stderr, so
# a run watched for silence (the GPU pool kills a command that writes nothing for 3 minutes) sees it alive
_current = {"id": None, "t0": 0.0}


def _heartbeat_start():
    import threading
    import time
    # pytest captures file descriptors 1 and 2 while a test runs: write to a duplicate of the real stderr taken now
    fd = os.dup(2)

    def beat():
        while True:
            time.sleep(60)
            tid = _current["id"]
            if tid is not None and time.time() - _current["t0"] >= 55:
                os.write(fd, f"[tests] {tid} running for {time.time() - _current['t0']:.0f} s\n".encode())
    threading.Thread(target=beat, daemon=True).start()


def pytest_runtest_setup(item):
    import time
    _current["id"], _current["t0"] = item.nodeid, time.time()


def pytest_runtest_teardown(item):
    _current["id"] = None


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def golden():
    return load_golden


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
