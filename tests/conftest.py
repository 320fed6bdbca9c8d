import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import psx  # noqa: E402,F401  (registers the package alias)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu on a GPU box")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _reset_deterministic(request):
    """The kernel library's deterministic-mode state is process-wide (an engine step sets it):
    every GPU test starts and ends with it off, so no test inherits another's mode."""
    if "gpu" not in request.keywords:
        yield
        return
    from psx.ops import kernels as K

    K.set_deterministic(None)
    yield
    K.set_deterministic(None)


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
