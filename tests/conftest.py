import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def built_lib():
    from reporter_amd import build
    build.build()
    build.build_oracle()
    return build.LIB


@pytest.fixture(scope="session")
def tmpdir_session(tmp_path_factory):
    return tmp_path_factory.mktemp("rm")


@pytest.fixture(scope="session")
def small_world(built_lib, tmpdir_session):
    """C1-sized graph (40x40 @100 m) shared by the tests."""
    from reporter_amd import world
    path = str(tmpdir_session / "c1.rmg")
    world.build_world(path, 40, 40, 100.0, seed=1)
    return path
