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


@pytest.fixture(scope="session")
def glossy_floor_obj():
    """modified_phong sphere and short box (CornellBox-Glossy.mtl: Ks 0.9 / 0.8, Ns 40)."""
    return os.path.join(SCENES, "CornellBox-Glossy-Floor.obj")


@pytest.fixture(scope="session")
def sphere_obj():
    """Two modified_phong spheres (Ns 1024): near-mirror lobes."""
    return os.path.join(SCENES, "CornellBox-Sphere.obj")


@pytest.fixture(scope="session")
def mirror_obj():
    return os.path.join(SCENES, "CornellBox-Mirror.obj")


@pytest.fixture(scope="session")
def glass_obj(tmp_path_factory):
    """Synthetic: CornellBox-Sphere with the right sphere at opacity 0.5, which
    mesh_loader.cpp:84-90 maps to dielectric(Ni 1.5).  No reference MTL has
    opacity < 1, so this is how a whole scene exercises the dielectric path."""
    d = tmp_path_factory.mktemp("glass")
    with open(os.path.join(SCENES, "CornellBox-Sphere.obj")) as f:
        obj = f.read().replace("mtllib CornellBox-Sphere.mtl", "mtllib CornellBox-Glass.mtl")
    with open(d / "CornellBox-Glass.obj", "w") as f:
        f.write(obj)
    out, cur = [], None
    with open(os.path.join(SCENES, "CornellBox-Sphere.mtl")) as f:
        for line in f:
            if line.startswith("newmtl"):
                cur = line.split()[1]
            if cur == "rightSphere" and line.startswith("Ni "):
                line = "Ni 1.5\nd 0.5\n"
            out.append(line)
    with open(d / "CornellBox-Glass.mtl", "w") as f:
        f.write("".join(out))
    return str(d / "CornellBox-Glass.obj")
