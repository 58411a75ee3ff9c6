"""Diagnostic A/B of the uniform decode kernel's roles (not part of the bench).

IGGY_CODEC_DBG bits (read at context creation): 1 = consumer skips the serial
batch-checksum chain, 32 = LDS-staged producers, 64 = lane-group producers stage
only (no hashing), 128 = lane-group producers publish nothing. DIAG_VARIANTS
selects the set (default 0,1,65,32).
All variants run interleaved in one process on the same batch.
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from iggy_amd import abi  # noqa: E402
from iggy_amd import codec as _codec  # noqa: E402

_codec.use_library(os.environ.get("IGGY_DIAG_LIB", _codec.DIAG_LIB_PATH))  # ablation bits: diagnostic build only
from iggy_amd.codec import Codec  # noqa: E402
import bench  # noqa: E402
from iggy_amd.torch_io import to_host  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    pl = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    variants = [int(v) for v in os.environ.get("DIAG_VARIANTS", "0,1,65,32").split(",")]
    ctxs = {}
    for v in variants:
        os.environ["IGGY_CODEC_DBG"] = str(v)
        ctxs[v] = Codec(0)
    os.environ.pop("IGGY_CODEC_DBG")
    ts = torch.cuda.Stream()
    torch.cuda.set_stream(ts)
    stream = ts.cuda_stream
    assert stream != 0
    batch = bench.make_batch(next(iter(ctxs.values())), n, pl, pl, 0, dev, stream)[0]
    L = batch.numel()
    if os.environ.get("DIAG_HIPMALLOC"):  # the record in a plain hipMalloc buffer instead of torch's allocator
        hip = ctypes.CDLL("libamdhip64.so")
        ptr = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(L + 4096)) == 0
        torch.cuda.synchronize()
        assert hip.hipMemcpy(ptr, ctypes.c_void_p(batch.data_ptr()), ctypes.c_size_t(L), 3) == 0  # D2D

        class _Rec:
            def __init__(self, p, n):
                self.p, self.n = p, n

            def data_ptr(self):
                return self.p

            def numel(self):
                return self.n

        del batch
        batch = _Rec(ptr.value, L)
        print(f"record at hipMalloc {ptr.value:#x}", flush=True)
    d_pos = torch.empty(n, dtype=torch.int64, device=dev)
    nopos = bool(os.environ.get("DIAG_NOPOS"))  # no frame-position output (the producers store none)
    pos_ptr, pos_cap = (None, 0) if nopos else (d_pos.data_ptr(), n)
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    for v, cx in ctxs.items():
        cx.reserve(L)
    res = {v: [] for v in variants}
    for integ in (0, 1):
        for rnd in range(3):
            for v, cx in ctxs.items():
                if integ == 1 and v != variants[0]:
                    continue
                for _ in range(2):
                    rc = cx.decode_device(batch.data_ptr(), L, integ, pos_ptr, pos_cap, d_res.data_ptr(), stream)
                    assert rc == 0, rc
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                d_res.zero_()
                for _ in range(10):
                    rc = cx.decode_device(batch.data_ptr(), L, integ, pos_ptr, pos_cap, d_res.data_ptr(), stream)
                    assert rc == 0, rc
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                r = abi.DecodeResult.from_buffer_copy(to_host(d_res).tobytes())
                print(f"integ={integ} dbg={v} round={rnd} ms={ms:.4f} GiB/s={L/ms/1e-3/2**30:.1f} "
                      f"err={r.error.kind} frames={r.frame_count} path={r.path}", flush=True)
                if v & 512 and rnd == 2 and integ == 0:  # progress stamps (10 ns ticks) of one more decode
                    L_ = cx._L
                    L_.iggy_codec_debug_clear.argtypes = [ctypes.c_void_p]
                    L_.iggy_codec_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
                    assert L_.iggy_codec_debug_clear(cx._h) == 0
                    rc = cx.decode_device(batch.data_ptr(), L, integ, pos_ptr, pos_cap, d_res.data_ptr(), stream)
                    buf = (ctypes.c_uint64 * 96)()
                    assert L_.iggy_codec_debug_read(cx._h, buf, 768) == 0
                    for gw in range(4):
                        npass, npoll, twait, tend = list(buf)[64 + 4 * gw: 68 + 4 * gw]
                        print(f"  gatherer {gw}: passes {npass} polls {npoll} ring-wait {twait / 100:.1f} us"
                              f" end {tend / 100:.1f} us", flush=True)
                    st = list(buf)[32:64]
                    t0 = st[0]
                    rel = lambda x: f"{(x - t0) / 100:.1f}" if x else "-"  # noqa: E731
                    print("  chain  batch 0,8,..: " + " ".join([rel(st[1])] + [rel(x) for x in st[3:10]])
                          + f"  done {rel(st[20])}  producers exited {rel(st[21])}", flush=True)
                    print("  staged batch 0,8,..: " + " ".join(rel(x) for x in st[23:31]), flush=True)
                    print("  blocks 0,1 published: " + " ".join(rel(x) for x in st[11:13])
                          + "  WG 0 steps 0-3 landed: " + " ".join(rel(x) for x in st[13:17]), flush=True)


if __name__ == "__main__":
    main()
