import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box via gpurun)")


def pytest_report_header(config):
    from dpwa_amd import _lib
    return "native library: %s" % _lib.LIB_PATH


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
