"""BASELINE config C4: end-to-end encode -> decode including pinned host<->device
copies, 262,144-message x 1 KiB batches streamed back-to-back.

Per batch (the path starts and ends in host memory):
  host SoA (ids, origin timestamps, payload bytes, lengths; pinned)
    --H2D--> encode_device --D2H--> wire bytes in pinned host memory (the "socket")
    --H2D--> decode_device(Verify) --D2H--> frame positions + result (the segment index)

Two modes:
  streams : two contexts on two streams alternate whole batches (round 1).
  async   : the product's asynchronous host API. The producer context encodes
            (iggy_codec_encode_submit: H2D of the SoA on its copy-in stream, the
            kernels, D2H of the wire bytes on its copy-out stream) and the server
            context decodes each finished batch (iggy_codec_decode_submit), so the
            two copy directions and the kernels of different batches overlap
            (full duplex on the link).
Reports the end-to-end GiB/s (batch bytes / wall time), the PCIe bytes moved,
and each phase's share measured on an isolated batch. Writes one JSON line
(recorded in DESIGN.md; never the bench `value`).
"""
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
from iggy_amd.codec import Codec  # noqa: E402

N = 262_144
PL = 1024


class Lane:
    """One context + stream + its device/pinned buffers."""

    def __init__(self, dev, n, pl):
        self.cx = Codec(dev.index or 0)
        self.s = torch.cuda.Stream(dev)
        self.n, self.pl = n, pl
        total = 256 + n * (48 + pl)
        self.total = total
        self.cx.reserve(total)
        self.d_ids = torch.empty(2 * n, dtype=torch.int64, device=dev)
        self.d_ots = torch.empty(n, dtype=torch.int64, device=dev)
        self.d_pay = torch.empty(n * pl, dtype=torch.uint8, device=dev)
        self.d_pls = torch.empty(n, dtype=torch.int32, device=dev)
        self.d_wire = torch.empty(total, dtype=torch.uint8, device=dev)
        self.d_wire2 = torch.empty(total, dtype=torch.uint8, device=dev)
        self.d_eres = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device=dev)
        self.d_pos = torch.empty(n, dtype=torch.int64, device=dev)
        self.d_dres = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
        self.h_wire = torch.empty(total, dtype=torch.uint8).pin_memory()
        self.h_pos = torch.empty(n, dtype=torch.int64).pin_memory()
        self.h_dres = torch.empty(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8).pin_memory()

    def run(self, src, timings=None):
        """Enqueue one whole batch on this lane's stream."""
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)] if timings is not None else None
        with torch.cuda.stream(self.s):
            if ev: ev[0].record()
            self.d_ids.copy_(src["ids"], non_blocking=True)
            self.d_ots.copy_(src["ots"], non_blocking=True)
            self.d_pay.copy_(src["pay"], non_blocking=True)
            self.d_pls.copy_(src["pls"], non_blocking=True)
            if ev: ev[1].record()
            raw = abi.RawMessages(self.n, self.d_ids.data_ptr(), self.d_ots.data_ptr(), self.d_pay.data_ptr(),
                                  self.d_pls.data_ptr(), None, None)
            rc = self.cx.encode_device(raw, 1, self.d_wire.data_ptr(), self.total, self.d_eres.data_ptr(),
                                       self.s.cuda_stream)
            assert rc == 0, rc
            if ev: ev[2].record()
            self.h_wire.copy_(self.d_wire, non_blocking=True)      # to the "socket"
            self.d_wire2.copy_(self.h_wire, non_blocking=True)     # server side receives it
            if ev: ev[3].record()
            rc = self.cx.decode_device(self.d_wire2.data_ptr(), self.total, abi.INTEGRITY_VERIFY,
                                       self.d_pos.data_ptr(), self.n, self.d_dres.data_ptr(), self.s.cuda_stream)
            assert rc == 0, rc
            if ev: ev[4].record()
            self.h_pos.copy_(self.d_pos, non_blocking=True)
            self.h_dres.copy_(self.d_dres, non_blocking=True)
            if ev: ev[5].record()
        if ev:
            self.s.synchronize()
            names = ["h2d_soa", "encode", "wire_d2h_h2d", "decode", "d2h_out"]
            for i, nm in enumerate(names):
                timings[nm] = ev[i].elapsed_time(ev[i + 1])

    def check(self):
        r = abi.DecodeResult.from_buffer_copy(self.h_dres.numpy().tobytes())
        assert r.error.kind == 0 and r.frame_count == self.n, r.error
        assert int(self.h_pos[1]) == 48 + self.pl


def run_async(src, n, batches):
    """Producer context encodes, server context decodes, through submit / wait."""
    import numpy as np
    from iggy_amd.codec import raw_messages
    A, B = Codec(0), Codec(0)
    total = 256 + n * (48 + PL)
    ids, ots, pay, pls = (src[k].numpy() for k in ("ids", "ots", "pay", "pls"))
    raw = raw_messages(ids.view(np.uint64), ots.view(np.uint64), pay, pls.view(np.uint32))
    wires = [torch.empty(total, dtype=torch.uint8).pin_memory().numpy() for _ in range(3)]
    poss = [torch.empty(n, dtype=torch.int64).pin_memory().numpy().view(np.uint64) for _ in range(3)]

    def once():
        te, td = {}, {}
        for b in range(batches + 2):
            if b < batches:
                te[b] = A.encode_submit(raw, 1, wires[b % 3])
            if 1 <= b <= batches:
                c = A.wait(te[b - 1])
                assert c.error.kind == 0 and c.bytes == total, c.error
                td[b - 1] = B.decode_submit(wires[(b - 1) % 3], abi.INTEGRITY_VERIFY, poss[(b - 1) % 3])
            if b >= 2:
                c = B.wait(td[b - 2])
                assert c.error.kind == 0 and c.frame_count == n, c.error
        assert int(poss[0][1]) == 48 + PL

    once()  # warm: slots and scratch sized
    t0 = time.perf_counter()
    once()
    wall = time.perf_counter() - t0
    A.close()
    B.close()
    return wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--messages", type=int, default=N)
    ap.add_argument("--mode", choices=["streams", "async"], default="async")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = args.messages
    g = torch.Generator().manual_seed(0x16619E3779B97F4A)
    src = {
        "ids": torch.randint(1, 2**62, (2 * n,), dtype=torch.int64, generator=g).pin_memory(),
        "ots": (1_700_000_000_000_000 + torch.arange(n, dtype=torch.int64)).pin_memory(),
        "pay": torch.randint(0, 256, (n * PL,), dtype=torch.uint8, generator=g).pin_memory(),
        "pls": torch.full((n,), PL, dtype=torch.int32).pin_memory(),
    }
    if args.mode == "async":
        wall_async = run_async(src, n, args.batches)
    lanes = [Lane(dev, n, PL), Lane(dev, n, PL)]
    # warm + isolated phase timings
    for ln in lanes:
        ln.run(src)
        ln.s.synchronize()
        ln.check()
    phases = {}
    lanes[0].run(src, phases)
    lanes[0].check()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(args.batches):
        lanes[b % 2].run(src)
    torch.cuda.synchronize()
    wall_streams = time.perf_counter() - t0
    wall = wall_async if args.mode == "async" else wall_streams
    for ln in lanes:
        ln.check()
    batch_bytes = lanes[0].total
    soa = src["ids"].numel() * 8 + src["ots"].numel() * 8 + src["pay"].numel() + src["pls"].numel() * 4
    pcie_per_batch = soa + 2 * batch_bytes + n * 8 + ctypes.sizeof(abi.DecodeResult)
    copy_ms = phases["h2d_soa"] + phases["wire_d2h_h2d"] + phases["d2h_out"]
    total_ms = sum(phases.values())
    line = {
        "config": "C4: encode->decode incl. pinned H2D/D2H, %d msgs x %d B per batch, %d batches, mode %s"
                  % (n, PL, args.batches, args.mode),
        "streams_mode_e2e_gib_s": round(args.batches * lanes[0].total / wall_streams / 2**30, 3),
        "e2e_gib_s": round(args.batches * batch_bytes / wall / 2**30, 3),
        "ms_per_batch": round(wall / args.batches * 1e3, 3),
        "pcie_bytes_per_batch": pcie_per_batch,
        "pcie_gb_s": round(args.batches * pcie_per_batch / wall / 1e9, 2),
        "isolated_batch_ms": {k: round(v, 3) for k, v in phases.items()},
        "pcie_share_isolated": round(copy_ms / total_ms, 3),
        "batch_bytes": batch_bytes,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
