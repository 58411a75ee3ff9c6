import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# The suite runs with the HIP runtime's defaults: the round-4 override of on-the-fly
# pinning (GPU_PINNED_MIN_XFER_SIZE) is gone, and a stale one from the caller's
# environment is dropped before anything initialises the runtime.
os.environ.pop("GPU_PINNED_MIN_XFER_SIZE", None)

# Host-memory history of this test process (iggy_amd/csrc/host_ctx.hpp hostmem_log): every range the
# codec registers, maps or pins, and its release, with test boundaries between; the tail
# is attached to a failing test's report, so a fault can be checked against earlier
# pinned or mapped ranges without running anything again.
HOSTMEM_LOG = os.environ.setdefault("IGGY_CODEC_HOSTMEM_LOG",
                                    os.path.join("/tmp", f"iggy_hostmem_{os.getpid()}.log"))

# torch first: its bundled HIP runtime then serves the codec library too (same
# sonames; see iggy_amd/codec.py load())
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


# Hot-path parity first: under -x a failure in a §8(f) widening module (records,
# SDK, encryption) must not hide the core decode/encode parity suite, which would
# otherwise sort after it alphabetically.
_MODULE_ORDER = ["test_parity_gpu", "test_configs_gpu", "test_robust_gpu", "test_convert_gpu",
                 "test_records_gpu", "test_sdk_gpu", "test_pollbody_gpu", "test_crypt_gpu", "test_hostmem_gpu"]


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        mod = item.module.__name__.rsplit(".", 1)[-1] if item.module else ""
        return _MODULE_ORDER.index(mod) if mod in _MODULE_ORDER else len(_MODULE_ORDER)
    items.sort(key=rank)  # stable: file order is kept inside a module


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


def _hostmem_mark(text):
    import time
    try:
        with open(HOSTMEM_LOG, "a") as f:
            f.write(f"{time.monotonic():.6f} test {text}\n")
    except OSError:
        pass


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_makereport(item, call):
    if call.when == "setup":
        _hostmem_mark(f"start {item.nodeid}")
    outcome = yield
    rep = outcome.get_result()
    if rep.failed and item.get_closest_marker("gpu") is not None:
        try:
            with open(HOSTMEM_LOG) as f:
                tail = f.readlines()[-60:]
        except OSError:
            tail = []
        if tail:
            rep.sections.append(("codec host-memory history (last 60 events)", "".join(tail)))
