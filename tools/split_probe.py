#!/usr/bin/env python3
"""Feasibility probe for hashing one host batch on the GPU and the CPU drop-in at once: C2's
1,024 x 8 MiB parts in pinned memory, the first m parts on the CPU route (sha256_batch_routed
route="cpu", host threads) in one Python thread while the rest go through the GPU host path
(sha256_batch_host) in another (ctypes drops the GIL).  Median wall time of --reps calls per m
after a warm call; digests vs the all-GPU result.  One JSON line per m.

    python3 tools/split_probe.py [--ms 0,256,384,448,512,576,1024] [--reps 3]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="0,256,384,448,512,576,1024")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--parts", type=int, default=1024)
    a = ap.parse_args()
    import torch

    import s3client_amd as s3
    n, L = a.parts, 8 * MIB
    lens = np.full(n, L, dtype=np.uint64)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    dev = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    s3.generate_parts(dev, offs, lens, np.arange(n), 20241008)
    pinned = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(dev)
    del dev
    torch.cuda.empty_cache()
    want = s3.sha256_batch_host(s3.BufferParts(pinned, offs, lens))
    rc = 0
    for m in [int(x) for x in a.ms.split(",")]:
        cpu_parts = s3.BufferParts(pinned, offs[:m], lens[:m]) if m else None
        gpu_parts = s3.BufferParts(pinned, offs[m:], lens[m:]) if m < n else None
        out = {}

        def run_cpu():
            t0 = time.perf_counter()
            out["cpu"] = s3.sha256_batch_routed(cpu_parts, route="cpu")[0]
            out["cpu_s"] = time.perf_counter() - t0

        def run_gpu():
            t0 = time.perf_counter()
            out["gpu"] = s3.sha256_batch_host(gpu_parts)
            out["gpu_s"] = time.perf_counter() - t0

        def once():
            ths = [threading.Thread(target=f) for f, p in ((run_cpu, cpu_parts), (run_gpu, gpu_parts)) if p is not None]
            t0 = time.perf_counter()
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            return time.perf_counter() - t0

        once()
        ts, cs, gs = [], [], []
        for _ in range(a.reps):
            ts.append(once())
            cs.append(out.get("cpu_s", 0.0))
            gs.append(out.get("gpu_s", 0.0))
        got = np.concatenate([out[k] for k, use in (("cpu", m > 0), ("gpu", m < n)) if use])
        ok = bool(np.array_equal(got, want))
        rc |= not ok
        t = float(np.median(ts))
        print(json.dumps({"cpu_parts": m, "ms": round(1e3 * t, 1), "GiBps": round(n * L / 2**30 / t, 2),
                          "cpu_ms": round(1e3 * float(np.median(cs)), 1),
                          "gpu_ms": round(1e3 * float(np.median(gs)), 1), "digests_ok": ok}), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
