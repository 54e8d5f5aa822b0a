import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tests' / 'golden'))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP path through the C-ABI)')
    config.addinivalue_line('markers', 'slow: longer CPU cases')


@pytest.fixture(scope='session')
def golden_dir():
    return ROOT / 'tests' / 'golden'
