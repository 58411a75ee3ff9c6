"""Device copy rate at the C3 encode's size (2.23 GB out of 2.2 GB in): the bound a
read-once / write-once kernel meets on this box, for DESIGN §4.4. Times torch's own
device copy (aligned: the runtime's DtoD copy), a byte-shifted copy, and the plain
kernels of scripts/copy_kernel.hip (16-B grid-stride copies; nontemporal stores;
unaligned 16-B stores) at several grid sizes, with events on torch's current stream.
usage: python scripts/copy_bound.py   (build scripts/_copy_kernel.so first, see the .hip)"""
import ctypes
import json
import os
import torch

N = 2_230_000_000
dev = torch.device("cuda:0")
src = torch.empty(N + 64, dtype=torch.uint8, device=dev)
src.random_(0, 256)
dst = torch.empty(N + 64, dtype=torch.uint8, device=dev)
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_copy_kernel.so"))
L.copy_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                          ctypes.c_void_p]


def kern(v, wgs):
    def f():
        st = torch.cuda.current_stream().cuda_stream
        rc = L.copy_launch(src.data_ptr(), dst.data_ptr(), N, v, wgs, st)
        assert rc == 0, rc
    return f


cases = [("torch_aligned", lambda: dst[:N].copy_(src[:N])),
         ("torch_dst_plus_1", lambda: dst[1:N + 1].copy_(src[:N]))]
for wgs in (1024, 2048, 4096, 16384):
    cases += [(f"k_plain_{wgs}", kern(0, wgs)), (f"k_nt_{wgs}", kern(1, wgs)), (f"k_unaligned_{wgs}", kern(2, wgs))]
out = {}
for name, fn in cases:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = min(ts)
    out[name] = {"ms_min": round(ms, 4), "ms_med": round(sorted(ts)[len(ts) // 2], 4),
                 "rw_TBps": round(2 * N / ms / 1e9, 3)}
    print(name, out[name], flush=True)
ok = torch.equal(dst[1:N + 1][:1 << 20], src[:1 << 20])  # the last case ran: unaligned
print(json.dumps({"bytes_each_way": N, "unaligned_copy_exact_prefix": bool(ok), **out}))
