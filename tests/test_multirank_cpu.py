"""The N>1 bench path on CPU: world_size-2 gloo ranks, one independent partition
per rank (BASELINE config C5 shape, reduced), with the bench's own max-over-ranks
timing reduction and aggregate-throughput formula. The data path has no
collective; each rank's batch is checked against the oracle only."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    import bench
    from oracle import oracle as O

    # each rank owns partition rank+1 (bench.make_batch uses partition_id = rank + 1)
    rec = O.synth_batch(2000, 1024, 1024, 0, seed=0x16619E3779B97F4A ^ rank, partition_id=rank + 1)
    rc, e, h, frames = O.decode_batch_slice_with(rec, 0)
    elapsed = 1.0 + 0.5 * rank  # stand-in per-rank timings
    m = bench.max_over_ranks(elapsed, dist)
    val = bench.whole_job_gib_s(world, rec.size, 10, m)
    out[rank] = (rc, h.partition_id, h.batch_checksum, len(frames), m, val, rec.size)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_partitions_and_timing():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_rank_main, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="fork")
    r0, r1 = out[0], out[1]
    assert r0[0] == r1[0] == 0                      # both partitions decode cleanly
    assert (r0[1], r1[1]) == (1, 2)                 # independent partitions, one per rank
    assert r0[2] != r1[2]                           # different batches
    assert r0[3] == r1[3] == 2000
    assert r0[4] == r1[4] == 1.5                    # max over ranks
    assert r0[5] == pytest.approx(2 * r0[6] * 10 / 1.5 / 2**30)


def test_bench_launcher_world2_dry():
    """`bench.py --gpus 2` with no launcher starts two rank processes itself (gloo
    rendezvous on 127.0.0.1), times with barrier + max over ranks, and rank 0 alone
    prints one JSON line with n_gpus = 2 (dry mode: the codec and GPU are stubbed)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry", "--steps", "4",
                        "--warmup", "1"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["scaling"] == "weak"
    # max over ranks: rank 1's stand-in step (2 ms) sets the time
    assert d["ms_per_step"] >= 2.0
