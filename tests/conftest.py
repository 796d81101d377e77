import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("stark-pure-rust_amd", "oracle"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    return O.Oracle()


@pytest.fixture(scope="session")
def ctx():
    import stark_amd
    c = stark_amd.Context(0)
    yield c
    c.close()
