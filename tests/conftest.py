import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")
    config.addinivalue_line("markers", "last: run after every other test (a failure under -x stops nothing else)")


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=lambda it: it.get_closest_marker("last") is not None)  # stable: the rest keep their order


@pytest.fixture(scope="session")
def oracle():
    from oracle import binding

    binding.lib()
    return binding
