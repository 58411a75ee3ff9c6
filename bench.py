"""Benchmark: device-resident message-batch decode on MI355X (BASELINE.json metric).

Workload (BASELINE configs[1], "C2"): one canonical Iggy batch of 1,048,576
messages x 1 KiB payload per GPU (1,124,073,728 bytes), resident in HBM; one
step = decode_batch_slice_with(Verify) of that batch
(core/binary_protocol/src/batch.rs:391-506): every frame walked and
XXH3-verified, the batch checksum recomputed and compared, the blob-relative
position of every frame written out (8 B per frame).

Steps alternate over `--streams` (default 2) lanes per GPU: each lane is its own
codec context + HIP stream + device-resident record (a partition's consecutive
batches), and every step is one complete single-record decode through
iggy_codec_decode_batch_device. Two lanes let one batch's serial batch-checksum
tail overlap the next batch's streaming phase; the
single-stream rate is reported beside it (`config.single_stream_gib_s`), and
`roofline` prices one launch at a time.

Multi-GPU (BASELINE configs[4], "C5"): one rank per GPU, each with its own
independent partition's batch; no data-path collective (weak scaling). The
barrier + max-over-ranks timing (gloo, CPU tensors) is the only cross-rank
traffic. `--gpus N` without a launcher starts the N rank processes itself
(before anything touches a GPU); under torch.distributed.run the ranks come
from the environment.

At N = 1 the line also carries, timed in the same run:
  c3_encode / c3_decode  BASELINE configs[2]: 1 M messages, payloads U[64, 4096] B,
                         device-resident encode (segmented lane-group path) and the
                         Verify decode of its output (general walk);
  c1                     BASELINE configs[0] shapes (10 batches x 1000 x 256 B):
                         cpu_ref encode/decode and the GPU's per-batch latency
                         (iggy-bench itself needs a Rust toolchain: not run);
  c4                     BASELINE configs[3]: 262,144 x 1 KiB batches encode ->
                         decode end to end through the asynchronous host API
                         (pinned H2D/D2H included), PCIe share and overlap;
  cpu_baseline           the oracle's AVX2 restatement of the C2 decode on this
                         host's cores (1, 8, 16 and nproc threads; reported, not
                         optimised against). At N > 1 rank 0 adds a short sample
                         (1 thread and one per rank).

The synthetic batches are produced on the GPU by the codec's own encoder
(SendMessagesEncoder semantics, server-twin form with partition_id = rank+1):
random full-range payload bytes, random non-zero ids, origin timestamps
1.7e15 + i microseconds.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from iggy_amd.torch_io import to_device, to_host  # noqa: E402  (copies through pinned staging)

METRIC = "GiB/s device-resident message-batch decode, 1M msgs × 1KiB payload"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
N_MSG = 1 << 20
PAYLOAD = 1024


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--messages", type=int, default=N_MSG)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-extra", action="store_true", help="skip the c3 / c1 legs")
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--streams", type=int, default=2, help="decode lanes (contexts/streams) steps alternate over")
    ap.add_argument("--dry", action="store_true",
                    help="codec-free rehearsal of the launcher, barrier and max-over-ranks timing (no GPU)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int, argv: list[str]) -> int:
    """One rank process per GPU (the parent never touches a GPU: it only waits)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


# ------------------------------------------------------------- cross-rank
def max_over_ranks(x: float, dist) -> float:
    """The bench's only cross-rank traffic: max of a per-rank scalar over gloo (CPU
    tensors). No data-path collective exists: partitions are independent."""
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def whole_job_gib_s(world: int, batch_bytes: int, steps: int, elapsed: float) -> float:
    """Aggregate throughput: every rank decodes `steps` batches of `batch_bytes` (weak scaling)."""
    return world * batch_bytes * steps / elapsed / 2**30


# ------------------------------------------------------------- workloads
def make_batch(cx, n: int, pl_lo: int, pl_hi: int, rank: int, dev, stream: int):
    """A stamped-form batch (partition_id = rank + 1) encoded on the GPU by the codec
    itself from random SoA input; payload lengths U[pl_lo, pl_hi]."""
    import torch
    from iggy_amd import abi

    g = torch.Generator(device=dev)
    g.manual_seed(0x16619E3779B97F4A ^ rank)
    if pl_lo == pl_hi:
        pls = torch.full((n,), pl_lo, dtype=torch.int32, device=dev)
    else:
        pls = torch.randint(pl_lo, pl_hi + 1, (n,), dtype=torch.int32, device=dev, generator=g)
    total_pl = int(pls.sum().item())
    payload = torch.randint(0, 256, (total_pl,), dtype=torch.uint8, device=dev, generator=g)
    ids = torch.randint(1, 2**62, (2 * n,), dtype=torch.int64, device=dev, generator=g)
    ots = 1_700_000_000_000_000 + torch.arange(n, dtype=torch.int64, device=dev)
    total = 256 + 48 * n + total_pl
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    res = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device=dev)
    raw = abi.RawMessages(n, ids.data_ptr(), ots.data_ptr(), payload.data_ptr(), pls.data_ptr(), None, None)
    torch.cuda.synchronize(dev)  # the inputs were made on torch's stream, the encode runs on `stream`
    rc = cx.encode_device(raw, rank + 1, out.data_ptr(), total, res.data_ptr(), stream)
    if rc:
        raise RuntimeError(f"encode_device rc={rc}")
    torch.cuda.synchronize(dev)
    er = abi.EncodeResult.from_buffer_copy(to_host(res).tobytes())
    if er.error.kind != 0 or er.batch_length != total:
        raise RuntimeError(f"encode failed: {er.error!r}")
    return out, (raw, ids, ots, payload, pls, res), total_pl


def c3_leg(cx, dev, steps: int):
    """BASELINE configs[2]: 1 M messages, payloads U[64, 4096]: device-resident encode
    (with per-message checksums and the batch checksum) and the Verify decode of its
    output, each timed over `steps` back-to-back calls on one stream."""
    import torch
    from iggy_amd import abi

    n = N_MSG
    s = torch.cuda.Stream(dev)
    out, keep, total_pl = make_batch(cx, n, 64, 4096, 7, dev, s.cuda_stream)
    raw, _ids, _ots, _pay, _pls, res = keep
    L = out.numel()
    dres = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    pos = torch.empty(n, dtype=torch.int64, device=dev)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / steps

    enc_s = timed(lambda: cx.encode_device(raw, 8, out.data_ptr(), L, res.data_ptr(), s.cuda_stream))
    er = abi.EncodeResult.from_buffer_copy(to_host(res).tobytes())
    assert er.error.kind == 0 and er.batch_length == L, er.error
    dec_s = timed(lambda: cx.decode_device(out.data_ptr(), L, abi.INTEGRITY_VERIFY, pos.data_ptr(), n,
                                           dres.data_ptr(), s.cuda_stream))
    dr = abi.DecodeResult.from_buffer_copy(to_host(dres).tobytes())
    assert dr.error.kind == 0 and dr.frame_count == n, dr.error
    enc_alg = total_pl + 32 * n + L  # payload + ids/timestamps/lengths in, batch out
    dec_alg = L + 8 * n
    del out, keep, pos
    return (
        {"ms": round(enc_s * 1e3, 4), "gib_s": round(L / enc_s / 2**30, 2), "batch_bytes": L,
         "algorithmic_bytes": enc_alg, "achieved_gbs": round(enc_alg / enc_s / 1e9, 1),
         "frac": round(enc_alg / enc_s / 1e9 / HBM_PEAK_GBS, 4),
         "workload": "C3: SendMessagesEncoder::encode on device, 1,048,576 msgs, payloads U[64,4096] B"},
        {"ms": round(dec_s * 1e3, 4), "gib_s": round(L / dec_s / 2**30, 2), "batch_bytes": L,
         "algorithmic_bytes": dec_alg, "achieved_gbs": round(dec_alg / dec_s / 1e9, 1),
         "frac": round(dec_alg / dec_s / 1e9 / HBM_PEAK_GBS, 4), "path": int(dr.path),
         "workload": "C3 record: decode_batch_slice_with(Verify), variable frame sizes (general walk)"},
    )


def crypt_leg(cx, dev, rec, n: int, steps: int, cpu: bool):
    """the at-rest encryption re-encode (encrypt_batch_request /
    decrypt_batch_record) of the C2 record on device, each timed over `steps`
    back-to-back calls; the CPU baseline is OpenSSL's AES-256-GCM on 1 KiB sections
    (the crypto alone, a lower bound on the reference's per-message re-encode)."""
    import torch
    from iggy_amd import abi

    L = rec.numel()
    s = torch.cuda.Stream(dev)
    key = bytes(range(32))
    nonces = torch.randint(0, 256, (24 * n,), dtype=torch.uint8, device=dev)
    cap = L + 28 * n
    enc = torch.empty(cap, dtype=torch.uint8, device=dev)
    dec = torch.empty(L, dtype=torch.uint8, device=dev)
    res = torch.zeros(ctypes.sizeof(abi.CryptResult), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / steps

    enc_s = timed(lambda: cx.encrypt_batch_device(key, rec.data_ptr(), L, nonces.data_ptr(), enc.data_ptr(), cap,
                                                  res.data_ptr(), s.cuda_stream))
    r = abi.CryptResult.from_buffer_copy(to_host(res).tobytes())
    assert r.error.kind == 0 and r.out_len == cap, r.error
    dec_s = timed(lambda: cx.decrypt_batch_device(key, enc.data_ptr(), cap, dec.data_ptr(), L, res.data_ptr(),
                                                  s.cuda_stream))
    r = abi.CryptResult.from_buffer_copy(to_host(res).tobytes())
    assert r.error.kind == 0 and r.out_len == L, r.error
    assert torch.equal(dec, rec), "decrypt(encrypt(x)) != x"
    out = {"workload": "encrypt_batch_request / decrypt_batch_record on the C2 record (1,048,576 x 1 KiB), "
                       "AES-256-GCM per payload",
           "encrypt_ms": round(enc_s * 1e3, 3), "decrypt_ms": round(dec_s * 1e3, 3),
           "encrypt_gib_s": round(L / enc_s / 2**30, 2), "decrypt_gib_s": round(cap / dec_s / 2**30, 2),
           "round_trip_exact": True}
    if cpu:
        from oracle import oracle as O  # cpu_baseline leg only
        by = {}
        for t in (1, 8, 16):
            r = O.cpu_gcm_gib_s(t, 0.5, 1024)
            if r > 0:
                by[str(t)] = round(r, 3)
        out["cpu_openssl_gcm_gib_s"] = by
        out["cpu_note"] = ("OpenSSL EVP_aes_256_gcm seal of 1 KiB sections, no framing or re-hash; T workers "
                           "released by one barrier, stopped by one 0.5-s deadline")
    del enc, dec, nonces
    return out


def c1_leg(cx, dev, seconds: float):
    """BASELINE configs[0] shapes: 10 batches x 1000 msgs x 256 B. iggy-bench over
    TCP needs a Rust toolchain (absent): recorded as not run; cpu_ref (the oracle's
    restatement, 1 thread) and the GPU's per-batch latency on the same shapes."""
    import torch
    from iggy_amd import abi
    from iggy_amd.codec import host_buffer, page_aligned, raw_messages
    from oracle import oracle as O  # cpu_ref leg of the bench only

    nb, n, pl = 10, 1000, 256
    rng = np.random.default_rng(0x16619E3779B97F4A)
    raws, keep, recs = [], [], []
    for b in range(nb):
        # page-aligned host buffers: registered below, and registrations may not share a page
        ids = page_aligned(rng.integers(1, 2**63, size=2 * n, dtype=np.uint64))
        ots = page_aligned((1_700_000_000_000_000 + b * n + np.arange(n)).astype(np.uint64))
        pay = page_aligned(rng.integers(0, 256, size=n * pl, dtype=np.uint8))
        pls = page_aligned(np.full(n, pl, dtype=np.uint32))
        raws.append(raw_messages(ids, ots, pay, pls))
        keep.append((ids, ots, pay, pls))
        rc, e, out = O.encode_batch(raws[-1], 0)
        assert rc == 0
        recs.append(page_aligned(np.frombuffer(out, dtype=np.uint8)))
    wire = sum(r.size for r in recs)

    def cpu_rate(one):  # one(batch index, reps) -> seconds for reps passes over that batch
        reps, secs, passes = 16, 0.0, 0
        while secs < seconds / 2:
            secs += sum(one(b, reps) for b in range(nb))
            passes += reps
        return passes * wire / secs

    enc = cpu_rate(lambda b, reps: O.cpu_encode_bench(raws[b], 0, 1, reps)[0])
    dec = cpu_rate(lambda b, reps: O.cpu_decode_bench(recs[b], 1, reps)[0])
    # GPU: device-resident decode of each batch (latency-bound at 304 KB) and the
    # host round trip through the asynchronous API (H2D, decode, D2H), per batch
    s = torch.cuda.Stream(dev)
    drecs = [to_device(r, dev) for r in recs]
    dres = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    for _ in range(3):
        for d, r in zip(drecs, recs):
            cx.decode_device(d.data_ptr(), r.size, 0, None, 0, dres.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(10):
        for d, r in zip(drecs, recs):
            cx.decode_device(d.data_ptr(), r.size, 0, None, 0, dres.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize(dev)
    dev_us = (time.perf_counter() - t0) / (10 * nb) * 1e6
    # device-resident encode of each batch (SendMessagesEncoder::encode from SoA input in HBM)
    denc = []
    for (ids, ots, pay, pls), r in zip(keep, recs):
        t = [to_device(a.view(np.int64) if a.dtype == np.uint64 else a, dev) for a in (ids, ots, pay, pls)]
        out = torch.empty(r.size, dtype=torch.uint8, device=dev)
        eres = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device=dev)
        raw = abi.RawMessages(n, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), None, None)
        denc.append((raw, t, out, eres))
    torch.cuda.synchronize(dev)
    for _ in range(3):
        for raw, _t, out, eres in denc:
            cx.encode_device(raw, 0, out.data_ptr(), out.numel(), eres.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(10):
        for raw, _t, out, eres in denc:
            cx.encode_device(raw, 0, out.data_ptr(), out.numel(), eres.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize(dev)
    enc_us = (time.perf_counter() - t0) / (10 * nb) * 1e6
    for _raw, _t, _out, eres in denc:
        er = abi.EncodeResult.from_buffer_copy(to_host(eres).tobytes())
        assert er.error.kind == 0, er.error
    def host_pass():
        for group in (recs[:8], recs[8:]):  # at most 8 in flight per context
            for t in [cx.decode_submit(r, 0) for r in group]:
                cx.wait(t)

    host_pass()  # untimed: the slots' pinned staging is allocated on first use
    t0 = time.perf_counter()
    for _ in range(5):
        host_pass()
    host_us = (time.perf_counter() - t0) / (5 * nb) * 1e6
    # the synchronous host decode (iggy_codec_decode_batch: one k_decode_records launch
    # and a host-mapped flag), pageable records, then the same records registered
    # (iggy_codec_host_register: the kernel reads them in place, no H2D)
    poss = [host_buffer(r.size // 48 + 1, np.uint64) for r in recs]

    def sync_us(reps=20):
        for r, p in zip(recs, poss):
            rc, nf = cx.decode_batch_into(r, abi.INTEGRITY_VERIFY, p)
            assert rc == 0 and nf == n, (rc, nf)
        t = time.perf_counter()
        for _ in range(reps):
            for r, p in zip(recs, poss):
                cx.decode_batch_into(r, abi.INTEGRITY_VERIFY, p)
        return (time.perf_counter() - t) / (reps * nb) * 1e6

    # The same synchronous calls timed from C (scripts/c_loop.c), the way the native
    # caller makes them: the Python loop above also pays ctypes' per-call argument
    # building (about 2-3 us of each call), which no Rust caller of the C ABI does.
    c_loop = None
    c_loop_path = os.path.join(ROOT, "scripts", "_c_loop.so")
    if os.path.exists(c_loop_path):
        c_loop = ctypes.CDLL(c_loop_path)
        c_loop.c_loop_decode.restype = ctypes.c_double
        c_loop.c_loop_decode.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_int, ctypes.c_int, ctypes.c_int]

    def sync_c_us(reps=50):
        if c_loop is None:
            return None
        k = len(recs)
        P = ctypes.c_void_p * k
        U = ctypes.c_uint64 * k
        args = (ctypes.cast(cx._L.iggy_codec_decode_batch, ctypes.c_void_p), cx._h,
                P(*[r.ctypes.data for r in recs]), U(*[r.size for r in recs]), P(*[p.ctypes.data for p in poss]),
                U(*[p.size for p in poss]), U(*[n] * k), k, abi.INTEGRITY_VERIFY)
        assert c_loop.c_loop_decode(*args, 2) > 0
        ns = c_loop.c_loop_decode(*args, reps)
        assert ns > 0, ns
        return ns / 1e3

    submit_cpu = [0.0]

    def async_us(reps=5, with_pos=True):
        t = time.perf_counter()
        sub = 0.0
        for _ in range(reps):
            for lo in (0, 8):  # at most 8 in flight per context
                c0 = time.thread_time()
                tks = [cx.decode_submit(recs[b], abi.INTEGRITY_VERIFY, poss[b] if with_pos else None)
                       for b in range(lo, min(lo + 8, nb))]
                sub += time.thread_time() - c0
                for tk in tks:
                    c = cx.wait(tk)
                    assert c.error.kind == 0 and c.frame_count == n, c.error
        submit_cpu[0] = sub / (reps * nb) * 1e6
        return (time.perf_counter() - t) / (reps * nb) * 1e6

    # the producer side: iggy_codec_encode_submit of the same SoA batches from host
    # memory into host wire buffers, 8 in flight (the SDK's direct-send path)
    wires = [host_buffer(r.size) for r in recs]
    enc_cpu = [0.0]

    def encode_async_us(reps=5):
        t = time.perf_counter()
        sub = 0.0
        for _ in range(reps):
            for lo in (0, 8):
                c0 = time.thread_time()
                tks = [cx.encode_submit(raws[b], 0, wires[b]) for b in range(lo, min(lo + 8, nb))]
                sub += time.thread_time() - c0
                for tk in tks:
                    c = cx.wait(tk)
                    assert c.error.kind == 0 and c.bytes == wires[0].size, c.error
        enc_cpu[0] = sub / (reps * nb) * 1e6
        return (time.perf_counter() - t) / (reps * nb) * 1e6

    sync_pageable_us = sync_us()
    for a in recs + poss + wires + [x for kp in keep for x in kp]:
        cx.host_register(a)
    try:
        sync_registered_us = sync_us()
        sync_registered_c_us = sync_c_us()
        assert all(int(p[1]) == 48 + pl for p in poss)
        # the same synchronous calls with the context's resident decode service
        # (iggy_codec_service_start: no launch per call)
        cx.service_start()
        try:
            for p in poss:
                p[:] = 0
            sync_registered_svc_us = sync_us()
            sync_registered_svc_c_us = sync_c_us()
            assert all(int(p[1]) == 48 + pl for p in poss)
        finally:
            cx.service_stop()
        for p in poss:
            p[:] = 0
        async_us(1)
        async_registered_us = async_us()
        assert all(int(p[1]) == 48 + pl for p in poss)
        encode_async_us(1)
        enc_async_registered_us = encode_async_us()
        assert all(np.array_equal(w, r) for w, r in zip(wires, recs))
    finally:
        for a in recs + poss + wires + [x for kp in keep for x in kp]:
            cx.host_unregister(a)
    return {
        "workload": "C1 shapes: 10 batches x 1000 msgs x 256 B (iggy-bench over TCP not run: no Rust toolchain)",
        "iggy_bench": None,
        "cpu_ref_encode_gib_s": round(enc / 2**30, 3), "cpu_ref_decode_gib_s": round(dec / 2**30, 3),
        "cpu_ref_threads": 1,
        "gpu_device_decode_us_per_batch": round(dev_us, 1),
        "gpu_device_encode_us_per_batch": round(enc_us, 1),
        "gpu_host_roundtrip_us_per_batch": round(host_us, 1),
        "gpu_host_sync_us_per_batch": round(sync_pageable_us, 1),
        "gpu_host_sync_registered_us_per_batch": round(sync_registered_us, 1),
        "gpu_host_sync_registered_service_us_per_batch": round(sync_registered_svc_us, 1),
        # the two synchronous forms above, timed from C (scripts/c_loop.c): no ctypes per call
        "gpu_host_sync_registered_c_loop_us_per_batch": (round(sync_registered_c_us, 1)
                                                          if sync_registered_c_us is not None else None),
        "gpu_host_sync_registered_service_c_loop_us_per_batch": (round(sync_registered_svc_c_us, 1)
                                                                  if sync_registered_svc_c_us is not None else None),
        "gpu_host_async_registered_us_per_batch": round(async_registered_us, 1),
        "gpu_host_async_registered_submit_cpu_us_per_batch": round(submit_cpu[0], 1),
        "gpu_host_encode_async_registered_us_per_batch": round(enc_async_registered_us, 1),
        "gpu_host_encode_async_registered_submit_cpu_us_per_batch": round(enc_cpu[0], 1),
        "cpu_ref_encode_us_per_batch": round(recs[0].size / enc * 1e6, 1),
        "cpu_ref_decode_us_per_batch": round(recs[0].size / dec * 1e6, 1),
        "wire_bytes": wire,
        "sync_note": ("gpu_host_sync_*: iggy_codec_decode_batch (decode_batch_slice_with's synchronous shape) per "
                      "call; *_service_*: the same calls after iggy_codec_service_start (resident workgroups, no "
                      "launch per call; opt-in per context), the others launch one kernel per call"),
    }


def c4_leg(dev, batches: int):
    """BASELINE configs[3] (C4): end-to-end encode -> decode including the pinned
    host<->device copies, 262,144 x 1 KiB batches streamed back to back through the
    product's asynchronous host API. A producer context encodes each batch from host
    SoA input (iggy_codec_encode_submit: H2D of the SoA, the kernels, D2H of the wire
    bytes into registered host memory -- the socket side), a server context decodes
    every finished batch (iggy_codec_decode_submit: H2D of the wire bytes, Verify
    decode, D2H of the frame positions -- the segment side); copy-in, kernels and
    copy-out of different batches overlap. Reported beside it: the same batch's PCIe
    copies and kernels timed alone (HIP events), the PCIe share of the isolated
    batch, and the overlap factor (isolated sum / pipelined time per batch)."""
    import torch
    from iggy_amd import abi
    from iggy_amd.codec import Codec, raw_messages

    n, pl = 262_144, 1024
    total = 256 + n * (48 + pl)
    g = torch.Generator().manual_seed(0x16619E3779B97F4A)
    t_ids = torch.randint(1, 2**62, (2 * n,), dtype=torch.int64, generator=g).pin_memory()
    t_ots = (1_700_000_000_000_000 + torch.arange(n, dtype=torch.int64)).pin_memory()
    t_pay = torch.randint(0, 256, (n * pl,), dtype=torch.uint8, generator=g).pin_memory()
    t_pls = torch.full((n,), pl, dtype=torch.int32).pin_memory()
    raw = raw_messages(t_ids.numpy().view(np.uint64), t_ots.numpy().view(np.uint64), t_pay.numpy(),
                       t_pls.numpy().view(np.uint32))
    wires = [torch.empty(total, dtype=torch.uint8).pin_memory() for _ in range(3)]
    poss = [torch.empty(n, dtype=torch.int64).pin_memory() for _ in range(3)]
    A, B = Codec(dev.index or 0), Codec(dev.index or 0)

    def once():
        te, td = {}, {}
        for b in range(batches + 2):
            if b < batches:
                te[b] = A.encode_submit(raw, 1, wires[b % 3].numpy())
            if 1 <= b <= batches:
                c = A.wait(te[b - 1])
                assert c.error.kind == 0 and c.bytes == total, c.error
                td[b - 1] = B.decode_submit(wires[(b - 1) % 3].numpy(), abi.INTEGRITY_VERIFY,
                                            poss[(b - 1) % 3].numpy().view(np.uint64))
            if b >= 2:
                c = B.wait(td[b - 2])
                assert c.error.kind == 0 and c.frame_count == n, c.error
        assert int(poss[0][1]) == 48 + pl

    once()  # slots and scratch sized
    t0 = time.perf_counter()
    once()
    wall = time.perf_counter() - t0
    A.close()
    B.close()
    # the same batch's pieces alone on one stream: PCIe copies and device-resident kernels
    cx = Codec(dev.index or 0)
    s = torch.cuda.Stream(dev)
    d_ids, d_ots, d_pay, d_pls = (t.to(dev) for t in (t_ids, t_ots, t_pay, t_pls))
    d_wire = torch.empty(total, dtype=torch.uint8, device=dev)
    d_pos = torch.empty(n, dtype=torch.int64, device=dev)
    d_eres = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device=dev)
    d_dres = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    draw = abi.RawMessages(n, d_ids.data_ptr(), d_ots.data_ptr(), d_pay.data_ptr(), d_pls.data_ptr(), None, None)
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(7)]
    ms = {}
    for rep in range(3):
        with torch.cuda.stream(s):
            ev[0].record()
            for dst, src in ((d_ids, t_ids), (d_ots, t_ots), (d_pay, t_pay), (d_pls, t_pls)):
                dst.copy_(src, non_blocking=True)
            ev[1].record()
            assert cx.encode_device(draw, 1, d_wire.data_ptr(), total, d_eres.data_ptr(), s.cuda_stream) == 0
            ev[2].record()
            wires[0].copy_(d_wire, non_blocking=True)
            ev[3].record()
            d_wire.copy_(wires[0], non_blocking=True)
            ev[4].record()
            assert cx.decode_device(d_wire.data_ptr(), total, abi.INTEGRITY_VERIFY, d_pos.data_ptr(), n,
                                    d_dres.data_ptr(), s.cuda_stream) == 0
            ev[5].record()
            poss[0].copy_(d_pos, non_blocking=True)
            ev[6].record()
        s.synchronize()
        ms = {k: ev[i].elapsed_time(ev[i + 1]) for i, k in
              enumerate(["h2d_soa", "encode", "d2h_wire", "h2d_wire", "decode", "d2h_positions"])}
    cx.close()
    dr = abi.DecodeResult.from_buffer_copy(to_host(d_dres).tobytes())
    assert dr.error.kind == 0 and dr.frame_count == n, dr.error
    soa = 16 * n + 8 * n + n * pl + 4 * n
    pcie = soa + 2 * total + 8 * n + 2 * ctypes.sizeof(abi.DecodeResult)
    copy_ms = ms["h2d_soa"] + ms["d2h_wire"] + ms["h2d_wire"] + ms["d2h_positions"]
    iso_ms = sum(ms.values())
    per = wall / batches
    return {
        "workload": "C4: SoA -> encode_submit -> wire bytes (host) -> decode_submit(Verify) -> positions (host), "
                    f"{n} msgs x {pl} B per batch, {batches} batches back to back, registered host buffers",
        "e2e_gib_s": round(total / per / 2**30, 3),
        "ms_per_batch": round(per * 1e3, 3),
        "batch_bytes": total,
        "pcie_bytes_per_batch": pcie,
        "pcie_gb_s": round(pcie / per / 1e9, 2),
        "isolated_batch_ms": {k: round(v, 3) for k, v in ms.items()},
        "pcie_share_isolated": round(copy_ms / iso_ms, 3),
        "overlap_factor": round(iso_ms / (per * 1e3), 3),
    }


def cpu_baseline(seconds: float, threads=None):
    """The oracle's restatement of the same decode on host cores (bounded sample).

    The sample is a full C2-shaped record (not cache-resident: 1.05 GiB), each
    thread walking and verifying the whole record serially (the reference's
    execution model: one shard thread per batch); T threads decode independent
    walks of it concurrently, T = 1, 8 (one per partition, C5), 16 (this process's
    CPU share on the GPU box) and nproc (the CPUs this process may run
    on). `threads` overrides the counts (multi-GPU lines: a short sample)."""
    from oracle import oracle as O  # cpu_baseline leg: the only bench use of oracle/

    rec = O.synth_batch(N_MSG, PAYLOAD, PAYLOAD)
    nbytes = rec.size

    def rate(threads):
        reps, total_secs, total_reps = 1, 0.0, 0
        while total_secs < seconds:
            secs, cs = O.cpu_decode_bench(rec, threads, reps)
            if cs == 0:
                raise RuntimeError("cpu baseline decode failed")
            total_secs += secs
            total_reps += reps
        return threads * total_reps * nbytes / total_secs / 2**30

    share = min(16, os.cpu_count() or 1)
    try:
        nproc = len(os.sched_getaffinity(0))
    except AttributeError:
        nproc = os.cpu_count() or 1
    counts = threads or sorted({1, min(8, share), share, nproc})
    rates = {t: rate(t) for t in counts}
    share = min(share, max(counts))
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    del rec
    return {
        "value": round(rates[share], 3), "unit": "GiB/s", "cores": share, "kind": "port",
        "sample": f"{N_MSG} msgs x {PAYLOAD} B payload ({nbytes} B record, not cache-resident), "
                  f"decode_batch_slice_with(Verify) walked serially per thread, >= {seconds:.0f} s per "
                  f"thread count; oracle C restatement with AVX2 XXH3",
        "by_threads_gib_s": {str(t): round(v, 3) for t, v in rates.items()},
        "single_thread_gib_s": round(rates[1], 3), "cpu_model": model,
        "host_cpus_visible": os.cpu_count(), "nproc": nproc,
        "note": "value = the 16-thread rate (this process's CPU share on the GPU box); T = nproc "
                "threads share those cores with every other thread of the box",
        "avx2": bool(O.lib().oracle_has_avx2()),
    }


def pmc_traffic(n: int):
    """HBM bytes per decode from the committed rocprofv3 PMC summary (FETCH_SIZE of the
    producer kernel, x2 per MI355X_MICROARCH.md for gfx950) when it matches this config."""
    path = os.path.join(ROOT, "profiles", "pmc_fetch.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("messages") != n or d.get("payload") != PAYLOAD or "k_decode_uniform" not in d.get("kernel", ""):
        return None, None
    return d.get("hbm_bytes_per_decode"), d.get("source")


# --------------------------------------------------------------------- main
def run(args, world: int, rank: int, local: int, dist):
    import torch
    from iggy_amd import abi
    from iggy_amd.codec import Codec

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n = args.messages
    # Steps alternate over `--streams` lanes, each its own codec context, HIP stream
    # and device-resident C2 record (a partition's consecutive batches): every step
    # is one complete decode_batch_slice_with(Verify) of one 1 M x 1 KiB batch,
    # enqueued through the single-record device API; lanes let one batch's serial
    # batch-checksum tail overlap the next batch's streaming phase.
    lanes = []
    for li in range(args.streams):
        cx = Codec(local)
        ts = torch.cuda.Stream(dev)
        batch, _keep, _ = make_batch(cx, n, PAYLOAD, PAYLOAD, rank * 16 + li, dev, ts.cuda_stream)
        del _keep
        cx.reserve(batch.numel())
        lanes.append({
            "cx": cx, "stream": ts.cuda_stream, "batch": batch,
            "pos": torch.empty(n, dtype=torch.int64, device=dev),
            "res": torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev),
        })
    L = lanes[0]["batch"].numel()
    torch.cuda.synchronize(dev)

    def step(i):
        ln = lanes[i % len(lanes)]
        rc = ln["cx"].decode_device(ln["batch"].data_ptr(), L, abi.INTEGRITY_VERIFY, ln["pos"].data_ptr(), n,
                                    ln["res"].data_ptr(), ln["stream"])
        if rc:
            raise RuntimeError(f"decode_device rc={rc}")

    for i in range(max(args.warmup, len(lanes))):
        step(i)
    torch.cuda.synchronize(dev)
    for ln in lanes:
        res = abi.DecodeResult.from_buffer_copy(to_host(ln["res"]).tobytes())
        if res.error.kind != 0 or res.frame_count != n or res.path != 1:
            raise RuntimeError(f"decode check failed: {res.error!r} frames={res.frame_count} path={res.path}")
        pos = to_host(ln["pos"][:4]).tolist()
        assert pos == [i * (48 + PAYLOAD) for i in range(4)], pos

    def timed(stepper):
        """Exactly args.steps steps between a barrier + device sync on both sides; the
        max over ranks."""
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.steps):
            stepper(i)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if dist:
            dist.barrier()
        return max_over_ranks(el, dist)

    def check_lanes():  # every timed decode left a clean result
        for ln in lanes:
            res = abi.DecodeResult.from_buffer_copy(to_host(ln["res"]).tobytes())
            if res.error.kind != 0 or res.frame_count != n:
                raise RuntimeError(f"timed decode failed: {res.error!r}")

    # Two forms of the same K steps, each timed on its own: lanes alternating (one
    # batch's chain tail under the next batch's stream) and one launch at a time on one
    # stream. `value` is the pipelined form, fixed up front (a partition's consecutive
    # batches in flight together; choosing the better of two single noisy timings after
    # the fact would bias the line upward); both numbers are in the line.
    elapsed_pipe = timed(step)
    check_lanes()
    elapsed_single = timed(lambda i: step(0)) if len(lanes) > 1 else elapsed_pipe
    check_lanes()
    elapsed = elapsed_pipe
    form = "pipelined" if len(lanes) > 1 else "single"

    # roofline: the decode grid's own duration, one launch at a time on one
    # stream (HIP events on the launch stream, bracketing k_decode_uniform)
    cx = lanes[0]["cx"]
    cx.profile_enable(True)
    for _ in range(args.steps):
        step(0)
        torch.cuda.synchronize(dev)
    launches, total_ms = cx.profile_read(0)
    cx.profile_enable(False)
    k_ms = total_ms / max(launches, 1)
    alg_bytes = L + 8 * n  # read the record once + one 8-B frame position per message
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    single_gib_s = L * args.steps / elapsed_single / 2**30
    pipe_gib_s = L * args.steps / elapsed_pipe / 2**30

    extra = {}
    if world == 1 and not args.no_extra:
        for ln in lanes[1:]:  # free HBM held by the other lanes' records
            ln["batch"] = None
        torch.cuda.empty_cache()
        # The side legs (other BASELINE configs) never take the headline line down with
        # them: a leg that fails reports its error in its own field.
        def leg(name, fn):
            try:
                return fn()
            except Exception as ex:  # reported, not hidden: the field carries the failure
                torch.cuda.synchronize()
                return {"error": f"{type(ex).__name__}: {ex}"[:500]}

        extra["crypt_c2"] = leg("crypt_c2", lambda: crypt_leg(lanes[0]["cx"], dev, lanes[0]["batch"], n,
                                                              max(5, args.steps // 4), rank == 0 and not args.no_cpu))
        lanes[0]["batch"] = None
        torch.cuda.empty_cache()
        c3 = leg("c3", lambda: c3_leg(lanes[0]["cx"], dev, max(5, args.steps // 2)))
        extra["c3_encode"], extra["c3_decode"] = c3 if isinstance(c3, tuple) else (c3, c3)
        torch.cuda.empty_cache()
        extra["c1"] = leg("c1", lambda: c1_leg(lanes[0]["cx"], dev, args.cpu_seconds))
        torch.cuda.empty_cache()
        extra["c4"] = leg("c4", lambda: c4_leg(dev, 16))
    cpu = None
    if rank == 0 and not args.no_cpu:
        # N = 1: the full sample; N > 1: a short one (1 thread and one per rank) so the
        # scaling lines carry the CPU axis too without lengthening the run much
        try:
            cpu = cpu_baseline(args.cpu_seconds) if world == 1 else \
                cpu_baseline(min(args.cpu_seconds, 1.5), threads=sorted({1, world}))
        except Exception as ex:  # reported in the line, never silently dropped
            cpu = {"error": f"{type(ex).__name__}: {ex}"[:500]}

    traffic, traffic_src = pmc_traffic(n)
    value = whole_job_gib_s(world, L, args.steps, elapsed)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (GPU-encoded batches, random payload bytes)",
        "config": {
            "workload": "C2: decode_batch_slice_with(Verify) of one device-resident batch per GPU, "
                        "1,048,576 msgs x 1 KiB payload",
            "messages_per_gpu": n,
            "payload_bytes": PAYLOAD,
            "batch_bytes": L,
            "outputs": "frame positions (8 B/msg) + result struct",
            "parallelism": f"{world} independent partitions, one per GPU, no collective",
            "streams_per_gpu": len(lanes),
            "value_form": form,
            "single_stream_gib_s": round(single_gib_s, 2),
            "pipelined_gib_s": round(pipe_gib_s, 2),
            "per_gpu_gib_s": round(value / world, 2),
            "per_gpu_hbm_frac": round(value / world * 2**30 / 1e9 / HBM_PEAK_GBS, 4),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": "k_decode_uniform<true> (one persistent grid: lane-group producers + chain WG), "
                      "one launch at a time",
            "kernel_ms": round(k_ms, 4),
            "algorithmic_bytes": alg_bytes,
        },
        "cpu_baseline": cpu,
    }
    line.update(extra)
    for ln in lanes:
        ln["cx"].close()
    return line


def run_dry(args, world: int, rank: int, dist):
    """The launcher / barrier / max-over-ranks path with a CPU stand-in for a step
    (tests/test_multirank_cpu.py runs it at world 2 on a GPU-less host)."""
    def step(i):
        time.sleep(0.001 * (1 + rank))

    for i in range(args.warmup):
        step(i)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(elapsed, dist)
    L = 256 + args.messages * (48 + PAYLOAD)
    return {"metric": METRIC, "value": round(whole_job_gib_s(world, L, args.steps, elapsed), 2), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "dry run (no codec, no GPU)",
            "config": {"workload": "dry", "parallelism": f"{world} ranks"}}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world == 0 and args.gpus > 1:
        # no launcher: start one rank per GPU ourselves, before any GPU call here
        sys.exit(launch(args.gpus, argv))
    world = max(world, 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    line = run_dry(args, world, rank, dist) if args.dry else run(args, world, rank, local, dist)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
