#!/usr/bin/env python3
"""Every host-memory entry point at config 2's scale (1,024 x 8 MiB = 8 GiB), H2D included:
SHA-256, MD5, SHA-256 + MD5 and verification (s3h_*_batch_host, s3h_verify_batch_host) from
pinned and pageable memory, and file ranges (s3h_sha256_file_parts, s3h_sha256_md5_file_parts)
from a file in the page cache.  Median of --reps timed calls after one warm call each; every
call's digests are checked against the first SHA-256 / MD5 result (and verification must
report no mismatch).  One JSON object on stdout.

    python3 tools/host_entry_rates.py [--reps 3] [--parts 1024]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
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
    pageable = pinned.numpy().copy()
    del dev
    torch.cuda.empty_cache()
    gib = n * L / 2**30
    res = {"parts": n, "part_bytes": L, "reps": a.reps, "GiBps": {}, "errors": []}
    ref = {}

    def timed(name, fn, check):
        fn()  # warm: contexts, plans, staging
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = fn()
            ts.append(time.perf_counter() - t0)
        if not check(out):
            res["errors"].append(name)
        res["GiBps"][name] = round(gib / float(np.median(ts)), 2)
        print(name, res["GiBps"][name], file=sys.stderr, flush=True)

    def same(key):
        def chk(out):
            if key not in ref:
                ref[key] = out
            return np.array_equal(out, ref[key])
        return chk

    for src, buf in (("pinned", pinned), ("pageable", pageable)):
        parts = s3.BufferParts(buf, offs, lens)
        timed(f"sha256_{src}", lambda: s3.sha256_batch_host(parts), same("sha256"))
        timed(f"md5_{src}", lambda: s3.md5_batch_host(parts), same("md5"))
        timed(f"sha256_md5_{src}", lambda: np.concatenate(s3.sha256_md5_batch_host(parts), axis=1),
              lambda out: np.array_equal(out[:, :8], ref["sha256"]) and np.array_equal(out[:, 8:], ref["md5"]))
        timed(f"verify_sha256_{src}", lambda: s3.verify_batch_host(parts, ref["sha256"]),
              lambda m: not np.asarray(m).any())
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        path = os.path.join(td, "c2.bin")
        pageable.tofile(path)
        timed("sha256_file", lambda: s3.sha256_file_parts(path, offs, lens), same("sha256"))
        timed("sha256_md5_file", lambda: np.concatenate(s3.sha256_md5_file_parts(path, offs, lens), axis=1),
              lambda out: np.array_equal(out[:, :8], ref["sha256"]) and np.array_equal(out[:, 8:], ref["md5"]))
    print(json.dumps(res))
    return 1 if res["errors"] else 0


if __name__ == "__main__":
    sys.exit(main())
