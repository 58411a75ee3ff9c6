"""Diagnostic: which codec entry point leaves a non-success HIP status behind
(hipPeekAtLastError) for the caller's thread."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iggy_amd import abi  # noqa: E402
from iggy_amd.codec import Codec, raw_messages  # noqa: E402
from oracle import oracle as O  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipPeekAtLastError.restype = ctypes.c_int


def chk(what):
    print(f"{what:40s} last={hip.hipPeekAtLastError()}", flush=True)


cx = Codec(0)
chk("create")
rec = O.synth_batch(3000, 1024, 1024, seed=1)
rc, e, h, f = cx.decode_batch_slice_with(rec, 0)
chk("decode sync")
t = cx.decode_submit(rec, 0, np.zeros(3001, dtype=np.uint64))
chk("decode_submit")
c = cx.poll(t)
chk("poll (maybe pending)")
c = cx.wait(t) if c is None else c
chk("wait")
buf = np.empty(rec.size, dtype=np.uint8)
buf[:] = rec
cx.host_register(buf)
chk("host_register")
ts = [cx.decode_submit(buf, 0) for _ in range(8)]
chk("8 submits")
try:
    cx.decode_submit(buf, 0)
except Exception as ex:
    print("busy:", ex)
chk("busy")
for t in ts:
    cx.wait(t)
chk("waits")
cx.host_unregister(buf)
chk("host_unregister")
try:
    cx.poll(ts[0])
except Exception as ex:
    print("stale:", ex)
chk("stale poll")
rng = np.random.default_rng(1)
n = 3000
pls = rng.integers(64, 4097, size=n).astype(np.uint32)
ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
raw = raw_messages(ids, ots, pay, pls)
out = np.zeros(256 + 48 * n + int(pls.sum()), dtype=np.uint8)
cx.wait(cx.encode_submit(raw, 0, out))
chk("encode_submit")
small = np.zeros(100, dtype=np.uint8)
cx.wait(cx.encode_submit(raw, 0, small))
chk("encode_submit small")
import torch  # noqa: E402
print("torch device count", torch.cuda.device_count(), flush=True)
torch.cuda.init()
print("torch init ok", flush=True)
