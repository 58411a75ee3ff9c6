"""iggy_amd — MI355X-native message-batch codec for Apache Iggy.

The product is the HIP library iggy_amd/libiggy_codec.so behind the C ABI in
include/iggy_codec.h; iggy_amd.codec is its Python host binding.
"""

import os as _os

# HIP runtime setting for processes that hand PAGEABLE host buffers to HIP copies
# (torch's .to("cuda") / .cpu(), the codec's synchronous host entry points given
# unregistered memory): no transient pinning of pageable ranges -- such copies go
# through the runtime's own pinned staging instead. On this pool the runtime's
# on-the-fly pinning faulted (hipErrorIllegalAddress / "Memory Fault Error" inside a
# pageable H2D or D2H) once host ranges it had pinned were freed and their addresses
# reused by later allocations. Must be set before the HIP runtime
# initialises: import iggy_amd (or set it in the environment) before torch.
RUNTIME_ENV = {"GPU_PINNED_MIN_XFER_SIZE": "1048576"}  # MiB: never pin on the fly


def apply_runtime_env() -> None:
    for k, v in RUNTIME_ENV.items():
        _os.environ.setdefault(k, v)


apply_runtime_env()
