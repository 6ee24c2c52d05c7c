#!/usr/bin/env python3
"""Host batch path with many small ragged parts (the shape of an uploader hashing many small
objects): n parts of U[lo, hi] bytes packed in one host buffer (pinned or pageable), through
s3h_sha256_batch_host; median GiB/s of --reps calls after a warm one, digests vs the first
call and vs hashlib on a sample.  One JSON line per (source, n).  --big KxM puts K parts of
M MiB among them (an object's parts batched with many small objects).

    python3 tools/host_small_parts.py [--ns 20000,100000] [--lo 1024] [--hi 131072] [--reps 3] [--big 4x16]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="20000,100000")
    ap.add_argument("--lo", type=int, default=1024)
    ap.add_argument("--hi", type=int, default=128 << 10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--big", default="")
    ap.add_argument("--routes", default="gpu", help="comma list of gpu / auto / split / cpu")
    a = ap.parse_args()
    import torch

    import s3client_amd as s3
    rc = 0
    for n in [int(x) for x in a.ns.split(",")]:
        rng = np.random.default_rng(n)
        lens = rng.integers(a.lo, a.hi + 1, n).astype(np.uint64)
        if a.big:
            k, m = (int(x) for x in a.big.split("x"))
            lens[rng.choice(n, k, replace=False)] = m << 20
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        total = int(lens.sum())
        src = rng.integers(0, 256, total, dtype=np.uint8)
        for kind in ("pinned", "pageable"):
            buf = torch.empty(total, dtype=torch.uint8, pin_memory=(kind == "pinned"))
            buf.numpy()[:] = src
            parts = s3.BufferParts(buf, offs, lens)
            ref = s3.sha256_batch_host(parts)
            for route in a.routes.split(","):
                def call():
                    if route == "gpu":
                        return s3.sha256_batch_host(parts), "gpu"
                    return s3.sha256_batch_routed(parts, route=route)
                call()
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    out, taken = call()
                    ts.append(time.perf_counter() - t0)
                sample = rng.integers(0, n, 16)
                ok = bool(np.array_equal(out, ref)) and all(
                    out[i].tobytes().hex() == hashlib.sha256(src[int(offs[i]):int(offs[i] + lens[i])]).hexdigest()
                    for i in sample)
                rc |= not ok
                print(json.dumps({"source": kind, "parts": n, "big": a.big or None, "route": route, "taken": taken,
                                  "GiB": round(total / 2**30, 3),
                                  "GiBps": round(total / 2**30 / float(np.median(ts)), 2),
                                  "ms": round(1e3 * float(np.median(ts)), 2), "digests_ok": ok}), flush=True)
            del buf, parts
    return rc


if __name__ == "__main__":
    sys.exit(main())
