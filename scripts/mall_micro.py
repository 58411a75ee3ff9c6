"""Copy-then-hash feasibility for the C3 encode: is a chunk that a copy
kernel has just written read back from the Infinity Cache, and does a chunked
copy -> read pipeline over 2.23 GB on two streams take longer than the copy alone?
Times, with HIP events on the streams the kernels run on:
  cold   : one read of the whole 2.23 GB (after an unrelated 1-GB write), xor / hash form
  copy   : the chunked copies alone (one stream)
  serial : copy chunk k, then read chunk k (one stream); the reads' own time summed
  pipe   : copies on stream A, reads of chunk k on stream B after chunk k's event
usage: python scripts/mall_micro.py  (build scripts/_mall_micro.so first, see the .hip)"""
import ctypes
import json
import os
import torch

N = 2_230_000_000 // (1 << 20) * (1 << 20)
dev = torch.device("cuda:0")
src = torch.empty(N, dtype=torch.uint8, device=dev)
src.random_(0, 256)
dst = torch.empty(N, dtype=torch.uint8, device=dev)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
sink = torch.zeros(8, dtype=torch.int64, device=dev)
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_mall_micro.so"))
L.mm_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
L.mm_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
sA = torch.cuda.Stream()
sB = torch.cuda.Stream()


def copy(off, n, st):
    assert L.mm_copy(src.data_ptr() + off, dst.data_ptr() + off, n, min(n // 4096, 4096), st.cuda_stream) == 0


def read(off, n, h, st):
    assert L.mm_read(dst.data_ptr() + off, n, h, min(n // 32768 * 4, 4096) or 1, sink.data_ptr(), st.cuda_stream) == 0


def flush():
    junk.fill_(1)
    torch.cuda.synchronize()


def ev(st):
    e = torch.cuda.Event(enable_timing=True)
    e.record(st)
    return e


out = {}
copy(0, N, sA)
torch.cuda.synchronize()
for h in (0, 1):
    ts = []
    for _ in range(3):
        flush()
        a = ev(sA); read(0, N, h, sA); b = ev(sA); b.synchronize()
        ts.append(a.elapsed_time(b))
    out[f"cold_read_h{h}"] = {"ms": round(min(ts), 4), "TBps": round(N / min(ts) / 1e9, 3)}
    print(out[f"cold_read_h{h}"], flush=True)
for C in (16 << 20, 32 << 20, 64 << 20, 128 << 20):
    nch = N // C
    r = {}
    # copies alone
    ts = []
    for _ in range(3):
        flush()
        a = ev(sA)
        for k in range(nch):
            copy(k * C, C, sA)
        b = ev(sA); b.synchronize()
        ts.append(a.elapsed_time(b))
    r["copy_ms"] = round(min(ts), 4)
    for h in (0, 1):
        # serial: the reads' own time
        best = None
        for _ in range(3):
            flush()
            evs = []
            a = ev(sA)
            for k in range(nch):
                copy(k * C, C, sA)
                e0 = ev(sA); read(k * C, C, h, sA); e1 = ev(sA)
                evs.append((e0, e1))
            b = ev(sA); b.synchronize()
            tot = a.elapsed_time(b)
            rd = sum(x.elapsed_time(y) for x, y in evs)
            if best is None or tot < best[0]:
                best = (tot, rd)
        r[f"serial_h{h}_ms"] = round(best[0], 4)
        r[f"serial_h{h}_read_ms"] = round(best[1], 4)
        r[f"serial_h{h}_read_TBps"] = round(N / best[1] / 1e9, 3)
        # pipelined on two streams
        ts = []
        for _ in range(3):
            flush()
            a = ev(sA)
            sB.wait_event(a)
            for k in range(nch):
                copy(k * C, C, sA)
                e = ev(sA)
                sB.wait_event(e)
                read(k * C, C, h, sB)
            b = ev(sB); b.synchronize()
            ts.append(a.elapsed_time(b))
        r[f"pipe_h{h}_ms"] = round(min(ts), 4)
    out[f"chunk_{C >> 20}MiB"] = r
    print(C >> 20, r, flush=True)
print(json.dumps({"bytes": N, **out}))
