import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def scene_paths(name):
    cam = "camera.yml" if name == "c0_default" else "%s_camera.yml" % name
    world = "c0_world.yml" if name == "c0_default" else "%s_world.yml" % name
    return os.path.join(SCENES, world), os.path.join(SCENES, cam)


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import c_oracle
    c_oracle.build()
    return c_oracle


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raytracing_rb_amd import _abi
    _abi.load_library()          # the HIP library must load: no fallback
    return torch.device("cuda", 0)
