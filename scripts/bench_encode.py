"""BASELINE config C3: device-resident encode + per-message checksum, 1,048,576
messages with payload lengths uniform in [64, 4096] B (the length prefix-scan
path). One step = SendMessagesEncoder::encode of the whole batch
(core/binary_protocol/src/requests/messages/send_messages.rs:89-181) from
device-resident SoA input: frame placement, header write, payload copy,
per-frame XXH3 backpatch, batch checksum, batch header.

Algorithmic bytes per encode: sum(payload) + 32 N (id 16 + origin
timestamp 8 + two lengths 8) + batch_length. Prints one JSON line (recorded in
DESIGN.md; the headline bench.py line is the C2 decode)."""
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

if os.environ.get("IGGY_DIAG_LIB"):  # ablation bits (IGGY_CODEC_DBG) live only in the diagnostic build
    _codec.use_library(os.environ["IGGY_DIAG_LIB"])
from iggy_amd.codec import Codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--messages", type=int, default=1 << 20)
    ap.add_argument("--lo", type=int, default=64)
    ap.add_argument("--hi", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-check", action="store_true",
                    help="ablation runs (wrong bytes by design): time the encode only, no decode check")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cx = Codec(0)
    ts = torch.cuda.Stream(dev)
    torch.cuda.set_stream(ts)
    s = ts.cuda_stream
    n = args.messages
    g = torch.Generator(device=dev).manual_seed(0x16619E3779B97F4A)
    pls = torch.randint(args.lo, args.hi + 1, (n,), dtype=torch.int32, device=dev, generator=g)
    spl = int(pls.sum().item())
    pay = torch.randint(0, 256, (spl,), dtype=torch.uint8, device=dev, generator=g)
    ids = torch.randint(1, 2**62, (2 * n,), dtype=torch.int64, device=dev, generator=g)
    ots = 1_700_000_000_000_000 + torch.arange(n, dtype=torch.int64, device=dev)
    total = 256 + 48 * n + spl
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    res = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device=dev)
    raw = abi.RawMessages(n, ids.data_ptr(), ots.data_ptr(), pay.data_ptr(), pls.data_ptr(), None, None)

    def step():
        rc = cx.encode_device(raw, 0, out.data_ptr(), total, res.data_ptr(), s)
        if rc:
            raise RuntimeError(f"encode_device rc={rc}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    er = abi.EncodeResult.from_buffer_copy(res.cpu().numpy().tobytes())
    assert er.error.kind == 0 and er.batch_length == total, er.error
    if args.no_check:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        print(json.dumps({"encode_ms": round(ms, 4), "checked": False}), flush=True)
        return
    # the encoded record must decode and verify (general walk: variable frame sizes)
    cap = n
    d_pos = torch.empty(cap, dtype=torch.int64, device=dev)
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    cx.reserve(total)
    assert cx.decode_device(out.data_ptr(), total, 0, d_pos.data_ptr(), cap, d_res.data_ptr(), s) == 0
    torch.cuda.synchronize()
    dr = abi.DecodeResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
    assert dr.error.kind == 0 and dr.frame_count == n, dr.error
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t1 = time.perf_counter()
    for _ in range(args.steps):
        assert cx.decode_device(out.data_ptr(), total, 0, d_pos.data_ptr(), cap, d_res.data_ptr(), s) == 0
    torch.cuda.synchronize()
    dec = time.perf_counter() - t1
    alg = spl + 32 * n + total
    ms = el / args.steps * 1e3
    line = {
        "config": f"C3: encode {n} msgs x U[{args.lo},{args.hi}] B payload, device-resident SoA input",
        "batch_bytes": total, "encode_ms": round(ms, 4),
        "encode_gib_s": round(total / (ms * 1e-3) / 2**30, 2),
        "algorithmic_bytes": alg, "achieved_gb_s": round(alg / (ms * 1e-3) / 1e9, 1),
        "hbm_frac": round(alg / (ms * 1e-3) / 8e12, 4),
        "decode_verify_ms": round(dec / args.steps * 1e3, 4),
        "decode_verify_gib_s": round(total / (dec / args.steps) / 2**30, 2),
    }
    print(json.dumps(line), flush=True)
    cx.close()


if __name__ == "__main__":
    main()
