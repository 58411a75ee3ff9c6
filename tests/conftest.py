import os
import sys

import pytest

# torch first: its bundled HIP runtime then serves the codec library too (same
# sonames; see iggy_amd/codec.py load())
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")
    config.addinivalue_line("markers", "gpu_diag: needs a GPU and the diagnostic build (next-round candidates); "
                                       "run explicitly with -m gpu_diag, never part of -m gpu")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
