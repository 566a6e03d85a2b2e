import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "c-filestorage-server-and-client_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


@pytest.fixture(scope="session")
def vectors():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def dummyfiles():
    with open(os.path.join(GOLDEN, "dummyfiles.json")) as f:
        return json.load(f)


def committed_file_bytes(entry):
    """Input bytes of a reference fixture file: committed copy, or regenerated (all-zero files)."""
    if entry["committed"]:
        with open(os.path.join(GOLDEN, "dummyFiles", entry["path"].replace("/", "__")), "rb") as f:
            return f.read()
    if entry["all_zero"]:
        return bytes(entry["U"])
    return None
