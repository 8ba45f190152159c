import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the product library and the oracle once per session (make is incremental)."""
    lib = os.path.join(REPO, "uvhttp_amd", "lib", "libuvhttp_ws_amd.so")
    orc = os.path.join(REPO, "oracle", "_build", "libws_oracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        subprocess.run(["make", "-C", REPO, "-j4"], check=True, stdout=subprocess.DEVNULL)
    yield


@pytest.fixture(scope="session")
def known_answers():
    import json
    with open(os.path.join(TESTS, "golden", "reference_known_answers.json")) as f:
        return json.load(f)
