"""Copies between host numpy arrays and torch device tensors through pinned staging.

Plumbing for the Python callers of the codec that move their own buffers with torch
(the tests, smoke(), bench.py). The HIP runtime copies PAGEABLE host memory by page-
locking the caller's range on the fly (ROCclr, transfers above GPU_PINNED_MIN_XFER_SIZE).
On this pool that path faulted (hipErrorIllegalAddress inside a pageable copy) in rounds
3-5, once inside torch's own `.to("cuda")` with no codec call since the last stream
synchronisation. The codec never uses that path (host_mem.hpp put_host /
get_host stage pageable bytes through its own pinned chunks); these helpers keep the
callers' own copies off it too: a host memcpy into torch's pinned (hipHostMalloc) cache,
then a DMA from page-locked memory.
"""
from __future__ import annotations

import os

import numpy as np

# Diagnostics only: IGGY_TORCH_IO_PAGEABLE=1 restores torch's plain pageable copies (the
# path that faulted), to run the suite once under the round-5 conditions with the codec's
# host-memory history attached to any failure (tests/conftest.py).
_PAGEABLE = os.environ.get("IGGY_TORCH_IO_PAGEABLE") == "1"


def to_device(a, device="cuda"):
    """A device tensor holding a copy of the numpy array `a` (same dtype and shape)."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a))
    if _PAGEABLE:
        return t.to(device)
    p = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    p.copy_(t)
    return p.to(device)


def to_host(t) -> np.ndarray:
    """A numpy copy of tensor `t` (synchronous; the copy lands in pinned memory)."""
    import torch
    if t.device.type == "cpu":
        return t.numpy()
    if _PAGEABLE:
        return t.cpu().numpy()
    p = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    p.copy_(t)
    return p.numpy()
