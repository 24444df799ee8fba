import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libste.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _heartbeat():
    """STE_TEST_HEARTBEAT=1 (with pytest -s): a line to stderr every 60 s while a test runs, so a
    long CPU-oracle comparison is not mistaken for a hung GPU job by an output watchdog."""
    if os.environ.get("STE_TEST_HEARTBEAT") != "1":
        yield
        return
    import threading
    import time
    stop = threading.Event()

    def beat():
        t0 = time.time()
        while not stop.wait(60):
            print(f"[heartbeat] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
