import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session", autouse=True)
def _built_libraries():
    from genomeanonymizer_amd.build import build_host, build_oracle
    build_host()
    build_oracle()
    yield


@pytest.fixture(scope="session")
def hip_built():
    from genomeanonymizer_amd.build import build_hip
    return build_hip()
