import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-experiments_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device and the built libmtx.so")


@pytest.fixture(scope="session")
def small_scene():
    """Bedroom proxy at 2 % of the triangle budget (≈37 k triangles), 64x36 film."""
    from mtx import scene

    return scene.bedroom(width=64, height=36, scale=0.02, tex_res=64)


@pytest.fixture(scope="session")
def full_scene():
    """The benchmark's bedroom proxy: 1,832,004 triangles, 1280x720 film."""
    from mtx import scene

    return scene.bedroom()


@pytest.fixture(scope="session")
def oracle():
    import binding

    binding.build()
    return binding
