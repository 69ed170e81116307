import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
CORNELL_OBJ = os.path.join(SCENES, "CornellBox-Original.obj")
VEACH_OBJ = os.path.join(SCENES, "veach_mi.obj")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def cornell_obj():
    return CORNELL_OBJ


@pytest.fixture(scope="session")
def veach_obj():
    return VEACH_OBJ
