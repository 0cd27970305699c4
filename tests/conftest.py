import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtbgpu.so on cuda:0)")


@pytest.fixture(autouse=True)
def _device_drained(request):
    """After every GPU test: the whole device synchronized, so an asynchronous fault is reported in
    the teardown of the test that caused it (an error left on a stream the test never synchronized
    again would otherwise surface in a later, unrelated test)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch

    if torch.cuda.is_available():
        torch.cuda.synchronize()
