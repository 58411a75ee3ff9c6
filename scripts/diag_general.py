"""Phase clock of the variable-size (general) decode on a C3-shaped record.
Encodes N messages with payloads U[lo, hi] on the device, decodes them twice,
and prints the general kernel's per-phase ticks (100 MHz) and link counters.
usage: python scripts/diag_general.py [--messages N] [--lo A] [--hi B]"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from iggy_amd import abi  # noqa: E402
from iggy_amd import codec as _codec  # noqa: E402

_codec.use_library(os.environ.get("IGGY_DIAG_LIB", _codec.DIAG_LIB_PATH))  # ablation bits live only in the diagnostic build
from iggy_amd.codec import Codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--messages", type=int, default=1 << 20)
    ap.add_argument("--lo", type=int, default=64)
    ap.add_argument("--hi", type=int, default=4096)
    ap.add_argument("--integrity", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cx = Codec(0)
    s = cx.stream()
    n = args.messages
    g = torch.Generator(device=dev).manual_seed(7)
    pls = torch.randint(args.lo, args.hi + 1, (n,), dtype=torch.int32, device=dev, generator=g)
    spl = int(pls.sum().item())
    pay = torch.randint(0, 256, (spl,), dtype=torch.uint8, device=dev, generator=g)
    ids = torch.randint(1, 2**62, (2 * n,), dtype=torch.int64, device=dev, generator=g)
    ots = 1_700_000_000_000_000 + torch.arange(n, dtype=torch.int64, device=dev)
    total = 256 + 48 * n + spl
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    res = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device=dev)
    raw = abi.RawMessages(n, ids.data_ptr(), ots.data_ptr(), pay.data_ptr(), pls.data_ptr(), None, None)
    torch.cuda.synchronize()
    assert cx.encode_device(raw, 0, out.data_ptr(), total, res.data_ptr(), s) == 0
    d_pos = torch.empty(n, dtype=torch.int64, device=dev)
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    cx.reserve(total)
    buf = (ctypes.c_uint64 * 96)()
    cx._L.iggy_codec_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    for it in range(3):
        t0 = time.perf_counter()
        assert cx.decode_device(out.data_ptr(), total, args.integrity, d_pos.data_ptr(), n, d_res.data_ptr(), s) == 0
        cx._L.iggy_codec_debug_read(cx.handle, buf, 768)
        ms = (time.perf_counter() - t0) * 1e3
        dr = abi.DecodeResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
        st = list(buf[64:82])
        line = {"iter": it, "host_ms": round(ms, 3), "err": dr.error.kind, "frames": dr.frame_count,
                "phase_us": [round(st[i] / 100, 1) for i in range(1, 7)],
                "fast_steps": st[8], "summary_groups": st[9], "span_groups": st[10], "repaired_groups": st[11],
                "ntiles": st[12], "tile_bytes": st[13],
                "verify_loop_end_max_us": round(st[14] / 100, 1), "verify_short_end_max_us": round(st[16] / 100, 1),
                "chain_done_us": round(buf[64 + 18] / 100, 1)}
        rep = list(buf[84:96])
        line["repairs"] = [{"tile": rep[6 * k], "true_entry": rep[6 * k + 1], "pick": rep[6 * k + 2],
                            "old_cnt": rep[6 * k + 3], "old_exit": rep[6 * k + 4],
                            "new_cnt": rep[6 * k + 5] & 0xFFFFFFFF, "new_exit": rep[6 * k + 5] >> 32}
                           for k in range(min(2, st[11]))]
        nvw = st[17]
        if nvw:
            line["verify_loop_end_mean_us"] = round(st[15] / nvw / 100, 1)
        print(json.dumps(line), flush=True)
    cx.close()


if __name__ == "__main__":
    main()
