import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'marl-snake_amd'), os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device); run with -m gpu')
    config.addinivalue_line('markers', 'slow: long CPU test')


@pytest.fixture(scope='session')
def oracle():
    from oracle import snake_oracle
    snake_oracle.build()
    return snake_oracle
