"""C4 end-to-end diagnosis (not part of the bench): the bench's C4 pipeline (encode_submit
-> wait -> decode_submit -> wait, two contexts, 262,144 x 1 KiB per batch, torch-pinned
host buffers) run against several builds of the library, each in its own process, with
and without a HIP runtime setting; beside it the PCIe ceiling of the same traffic from
plain torch copies (H2D alone, D2H alone, both directions at once).

usage: python scripts/c4_diag.py --all [--libs a.so b.so ...]      (driver: one child per case)
       python scripts/c4_diag.py --lib X.so [--reps 3] [--torch]   (one case)
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def minimal_load(path):
    """Only the entry points the pipeline uses (older builds lack later symbols)."""
    import torch  # noqa: F401  (torch's HIP runtime first, as iggy_amd.codec.load does)
    vp, u64, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    L = ctypes.CDLL(path)
    L.iggy_codec_create.argtypes = [ci, ctypes.POINTER(vp)]
    L.iggy_codec_destroy.argtypes = [vp]
    L.iggy_codec_destroy.restype = None
    L.iggy_codec_decode_submit.argtypes = [vp, vp, u64, ci, vp, u64, ctypes.POINTER(u64)]
    L.iggy_codec_encode_submit.argtypes = [vp, vp, u64, vp, u64, ctypes.POINTER(u64)]
    L.iggy_codec_wait.argtypes = [vp, u64, vp]
    return L


def torch_ceiling(n_bytes, reps=3):
    import torch
    dev = torch.device("cuda", 0)
    h1 = torch.empty(n_bytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n_bytes, dtype=torch.uint8).pin_memory()
    h3 = torch.empty(n_bytes, dtype=torch.uint8).pin_memory()
    d1 = torch.empty(n_bytes, dtype=torch.uint8, device=dev)
    d2 = torch.empty(n_bytes, dtype=torch.uint8, device=dev)
    d3 = torch.empty(n_bytes, dtype=torch.uint8, device=dev)
    s = [torch.cuda.Stream(dev) for _ in range(3)]
    out = {}

    def run(name, ops):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for (dst, src), st in zip(ops, s):
                with torch.cuda.stream(st):
                    dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            best = dt if best is None else min(best, dt)
        out[name] = round(best, 3)

    run("h2d_ms", [(d1, h1)])
    run("d2h_ms", [(h1, d1)])
    run("h2d_and_d2h_ms", [(d1, h1), (h2, d2)])
    run("h2d_and_h2d_ms", [(d1, h1), (d2, h2)])
    run("2h2d_and_d2h_ms", [(d1, h1), (d2, h2), (h3, d3)])
    out["bytes_each"] = n_bytes
    return out


def pipeline(L, batches, reps):
    import numpy as np
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
    A, B = Codec(0, library=L), Codec(0, library=L)
    pinned = None
    if hasattr(L, "iggy_codec_host_pinned"):
        L.iggy_codec_host_pinned.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        pinned = {k: L.iggy_codec_host_pinned(t.data_ptr(), t.numel() * t.element_size())
                  for k, t in (("ids", t_ids), ("pay", t_pay), ("wire", wires[0]), ("pos", poss[0]))}

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

    once()
    per = []
    for _ in range(reps):
        t0 = time.perf_counter()
        once()
        per.append((time.perf_counter() - t0) / batches * 1e3)
    # encode alone, back to back (no decode context): its own overlap of H2D and D2H
    enc_only = []
    for _ in range(reps):
        t0 = time.perf_counter()
        tk = [A.encode_submit(raw, 1, wires[b % 3].numpy()) for b in range(3)]
        for b in range(3, batches):
            A.wait(tk[b - 3])
            tk.append(A.encode_submit(raw, 1, wires[b % 3].numpy()))
        for t in tk[-3:]:
            A.wait(t)
        enc_only.append((time.perf_counter() - t0) / batches * 1e3)
    A.close()
    B.close()
    return {"ms_per_batch": [round(x, 3) for x in per], "e2e_gib_s": round(total / (min(per) * 1e-3) / 2**30, 3),
            "encode_only_ms_per_batch": [round(x, 3) for x in enc_only], "host_pinned": pinned}


def child(args):
    import torch
    torch.cuda.set_device(0)
    rec = {"lib": os.path.relpath(args.lib, ROOT), "env": {k: os.environ[k] for k in ("GPU_PINNED_MIN_XFER_SIZE",)
                                                          if k in os.environ}}
    L = minimal_load(args.lib)
    rec.update(pipeline(L, args.batches, args.reps))
    if args.torch:
        rec["torch_ceiling"] = torch_ceiling(256 + 262_144 * 1072)
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--libs", nargs="*", default=None)
    ap.add_argument("--lib", default=os.path.join(ROOT, "iggy_amd", "libiggy_codec.so"))
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--envs", default="none,pin", help="comma list: none | pin (GPU_PINNED_MIN_XFER_SIZE=1048576)")
    args = ap.parse_args()
    if not args.all:
        return child(args)
    libs = args.libs or [os.path.join(ROOT, "iggy_amd", "libiggy_codec.so")]
    first = True
    for envname in args.envs.split(","):
        for lib in libs:
            env = dict(os.environ)
            env.pop("GPU_PINNED_MIN_XFER_SIZE", None)
            if envname == "pin":
                env["GPU_PINNED_MIN_XFER_SIZE"] = "1048576"
            cmd = [sys.executable, "-u", os.path.abspath(__file__), "--lib", lib, "--batches", str(args.batches),
                   "--reps", str(args.reps)] + (["--torch"] if first else [])
            first = False
            p = subprocess.run(cmd, env=env, timeout=240)
            if p.returncode != 0:
                print(json.dumps({"lib": lib, "env": envname, "rc": p.returncode}), flush=True)
                return p.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
