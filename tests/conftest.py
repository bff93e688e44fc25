import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "run_last: a code path with no GPU run behind it yet; runs after the rest")


def pytest_collection_modifyitems(config, items):
    """Tests marked run_last go to the end of the run (stable order
    otherwise): a fault in a path that has not run on a GPU before cannot
    cut the verified tests' run short."""
    items[:] = [i for i in items if i.get_closest_marker("run_last") is None] + \
               [i for i in items if i.get_closest_marker("run_last") is not None]


@pytest.fixture(scope="session")
def gpu():
    """One engine handle on cuda:0 for the GPU parity tests."""
    from cilium_amd.classifier import Classifier
    cl = Classifier(device=0)
    yield cl
    cl.close()


@pytest.fixture(scope="session")
def host():
    """A host-only handle (device=-1): compiles and packs, refuses verdicts."""
    from cilium_amd.classifier import Classifier
    cl = Classifier(device=-1)
    yield cl
    cl.close()
