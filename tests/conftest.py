import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


def pytest_collection_modifyitems(config, items):
    # Skip GPU tests only where there is no GPU device node at all (the CPU
    # container). On a GPU box a runtime that cannot see the GPU must FAIL the
    # tests (their fixtures assert), never silently skip them.
    if os.path.exists("/dev/kfd"):
        return
    skip = pytest.mark.skip(reason="no GPU device (/dev/kfd) on this host")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def orc():
    import oracle

    return oracle.Oracle()


def golden_blocks(entry, n, length):
    import numpy as np

    raw = np.fromfile(os.path.join(GOLDEN, entry["file"]), dtype=np.uint8)
    assert raw.size == n * length
    return [raw[i * length:(i + 1) * length] for i in range(n)]
