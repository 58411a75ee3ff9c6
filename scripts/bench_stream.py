"""Same-box A/B (diagnostic): the C3 decode (1 M msgs, U[64, 4096] B, Verify) by the
product general walk (libiggy_codec.so, decode_general.hip) and by the streamed
candidate (libiggy_codec_diag.so with dbg bit 0x200000, decode_stream.hip), both in
one process on the same device-resident record; each result checked (no error,
every frame). One JSON line per library."""
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
from iggy_amd.codec import DIAG_LIB_PATH, Codec, load, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--messages", type=int, default=1 << 20)
    ap.add_argument("--lo", type=int, default=64)
    ap.add_argument("--hi", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = args.messages
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    pls = torch.randint(args.lo, args.hi + 1, (n,), dtype=torch.int32, device=dev, generator=g)
    spl = int(pls.sum().item())
    pay = torch.randint(0, 256, (spl,), dtype=torch.uint8, device=dev, generator=g)
    ids = torch.randint(1, 2**62, (2 * n,), dtype=torch.int64, device=dev, generator=g)
    ots = 1_700_000_000_000_000 + torch.arange(n, dtype=torch.int64, device=dev)
    total = 256 + 48 * n + spl
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    eres = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device=dev)
    raw = abi.RawMessages(n, ids.data_ptr(), ots.data_ptr(), pay.data_ptr(), pls.data_ptr(), None, None)
    d_pos = torch.empty(n, dtype=torch.int64, device=dev)
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    prod = Codec(0, library=lib())
    s = torch.cuda.current_stream().cuda_stream
    assert prod.encode_device(raw, 0, out.data_ptr(), total, eres.data_ptr(), s) == 0
    torch.cuda.synchronize()
    os.environ["IGGY_CODEC_DBG"] = str(0x200000)
    diag = Codec(0, library=load(DIAG_LIB_PATH))
    del os.environ["IGGY_CODEC_DBG"]
    for name, cx in (("general (product)", prod), ("stream (diag 0x200000)", diag)):
        cx.reserve(total)
        for it in range(2 + args.steps):
            if it == 2:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            assert cx.decode_device(out.data_ptr(), total, 0, d_pos.data_ptr(), n, d_res.data_ptr(), s) == 0
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        dr = abi.DecodeResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
        print(json.dumps({"decoder": name, "ms": round(ms, 4), "gib_s": round(total / (ms * 1e-3) / 2**30, 1),
                          "frac": round((total + 8 * n) / (ms * 1e-3) / 8e12, 4), "err": dr.error.kind,
                          "frames": dr.frame_count, "path": dr.path, "ok": dr.error.kind == 0 and dr.frame_count == n}),
              flush=True)
    diag.close()
    prod.close()


if __name__ == "__main__":
    main()
