import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "binary-image-compression_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


def _ensure_built():
    # the checker (oracle/liboracle.so) is plain C: build it if this snapshot lacks it
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def oracle():
    _ensure_built()
    from oracle_lib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "golden.json")) as f:
        meta = json.load(f)
    arrays = np.load(os.path.join(g, "golden.npz"), allow_pickle=False)
    return meta, arrays


@pytest.fixture(scope="session")
def ctx():
    import pybic
    c = pybic.Context(0)  # raises if libbic.so or the gfx950 device is missing: no fallback
    yield c
    c.sync()
    c.close()
