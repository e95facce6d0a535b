import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "karpenter-provider-aws_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs through libkpsim.so")


@pytest.fixture(scope="session")
def fx():
    from kpsim import catalog
    return catalog.load_fixtures()


@pytest.fixture(scope="session")
def golden(fx):
    from kpsim import catalog
    return catalog.golden_catalog(fx=fx)


@pytest.fixture(scope="session")
def fake(fx):
    from kpsim import catalog
    return catalog.fake_catalog(fx=fx)
