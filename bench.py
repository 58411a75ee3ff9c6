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
barrier + max-over-ranks timing is the only cross-rank traffic.

The synthetic batches are produced on the GPU by the codec's own encoder
(SendMessagesEncoder semantics, server-twin form with partition_id = rank+1):
random full-range payload bytes, random non-zero ids, origin timestamps
1.7e15 + i microseconds.

Output: ONE JSON line on rank 0 with `roofline` (dominant kernel, HIP events
on the launch stream) and `cpu_baseline` (the oracle's AVX2 restatement of the
same decode timed on this host's cores; reported, not optimised against).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from iggy_amd import abi  # noqa: E402
from iggy_amd.codec import Codec  # noqa: E402

METRIC = "GiB/s device-resident message-batch decode, 1M msgs × 1KiB payload"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
N_MSG = 1 << 20
PAYLOAD = 1024


def make_batch(cx: Codec, n: int, pl: int, rank: int, dev: torch.device, stream: int):
    g = torch.Generator(device=dev)
    g.manual_seed(0x16619E3779B97F4A ^ rank)
    payload = torch.randint(0, 256, (n * pl,), dtype=torch.uint8, device=dev, generator=g)
    pls = torch.full((n,), pl, dtype=torch.int32, device=dev)
    ids = torch.randint(1, 2**62, (2 * n,), dtype=torch.int64, device=dev, generator=g)
    ots = 1_700_000_000_000_000 + torch.arange(n, dtype=torch.int64, device=dev)
    total = 256 + n * (48 + pl)
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    res = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device=dev)
    raw = abi.RawMessages(n, ids.data_ptr(), ots.data_ptr(), payload.data_ptr(), pls.data_ptr(), None, None)
    rc = cx.encode_device(raw, rank + 1, out.data_ptr(), total, res.data_ptr(), stream)
    if rc:
        raise RuntimeError(f"encode_device rc={rc}")
    torch.cuda.synchronize(dev)
    er = abi.EncodeResult.from_buffer_copy(res.cpu().numpy().tobytes())
    if er.error.kind != 0 or er.batch_length != total:
        raise RuntimeError(f"encode failed: {er.error!r}")
    del payload, pls, ids, ots
    return out


def cpu_baseline(n_sample: int, seconds: float):
    """The oracle's restatement of the same decode on host cores (bounded sample).

    The sample is a full C2-shaped record (not cache-resident: 1.05 GiB), each
    thread walking and verifying the whole record serially (the reference's
    execution model: one shard thread per batch); T threads decode independent
    walks of it concurrently."""
    from oracle import oracle as O  # cpu_baseline leg: the only bench use of oracle/

    rec = O.synth_batch(n_sample, PAYLOAD, PAYLOAD)
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

    threads = min(16, os.cpu_count() or 1)
    r1 = rate(1)
    rt = rate(threads)
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
        "value": round(rt, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": f"{n_sample} msgs x {PAYLOAD} B payload ({nbytes} B record, not cache-resident), "
                  f"decode_batch_slice_with(Verify) walked serially per thread, >= {seconds:.0f} s per "
                  f"thread count; oracle C restatement with AVX2 XXH3, -O3 -march=native",
        "single_thread_gib_s": round(r1, 3), "cpu_model": model,
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


def max_over_ranks(x: float, dist, device) -> float:
    """The bench's only cross-rank traffic: max of a per-rank scalar (RCCL on GPUs,
    gloo in the CPU tests). No data-path collective exists: partitions are independent."""
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def whole_job_gib_s(world: int, batch_bytes: int, steps: int, elapsed: float) -> float:
    """Aggregate throughput: every rank decodes `steps` batches of `batch_bytes` (weak scaling)."""
    return world * batch_bytes * steps / elapsed / 2**30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--messages", type=int, default=N_MSG)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--streams", type=int, default=2, help="decode lanes (contexts/streams) steps alternate over")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", init_method="env://")
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
        batch = make_batch(cx, n, PAYLOAD, rank * 16 + li, dev, ts.cuda_stream)
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
        res = abi.DecodeResult.from_buffer_copy(ln["res"].cpu().numpy().tobytes())
        if res.error.kind != 0 or res.frame_count != n or res.path != 1:
            raise RuntimeError(f"decode check failed: {res.error!r} frames={res.frame_count} path={res.path}")
        pos = ln["pos"][:4].cpu().tolist()
        assert pos == [i * (48 + PAYLOAD) for i in range(4)], pos

    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(elapsed, dist, dev)
    for ln in lanes:  # every timed decode left a clean result
        res = abi.DecodeResult.from_buffer_copy(ln["res"].cpu().numpy().tobytes())
        if res.error.kind != 0 or res.frame_count != n:
            raise RuntimeError(f"timed decode failed: {res.error!r}")

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
    # single-stream step rate, for reference (no overlap between batches)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step(0)
    torch.cuda.synchronize(dev)
    single_gib_s = L * args.steps / (time.perf_counter() - t1) / 2**30

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(N_MSG, args.cpu_seconds)

    traffic, traffic_src = pmc_traffic(n)
    ms_per_step = elapsed / args.steps * 1e3
    value = whole_job_gib_s(world, L, args.steps, elapsed)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
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
                "single_stream_gib_s": round(single_gib_s, 2),
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
        print(json.dumps(line), flush=True)
    for ln in lanes:
        ln["cx"].close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
