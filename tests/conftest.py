import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)
GOLDEN = os.path.join(HERE, 'golden')
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the C-ABI library)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


@pytest.fixture(scope='session')
def golden_fluxes():
    import json
    with open(os.path.join(GOLDEN, 'fluxes.json')) as f:
        return json.load(f)
