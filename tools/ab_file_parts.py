#!/usr/bin/env python3
"""A/B of the host path's file-range sources on one box, alternating: s3h_sha256_file_parts
with its automatic choice, forced pread slices (4 / 8 KiB = a 32 MiB staging slot at 8,192 /
4,096 parts, 32 KiB = a 128 MiB slot at 4,096), and pointers into a mapping the caller keeps (sha256_batch_host).
Usage: ab_file_parts.py FILE PARTS [REPS]; prints one JSON line per variant (median GiB/s)."""
import json
import mmap
import sys
import time

import numpy as np

import s3client_amd as s3


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    with open(path, "rb") as f:
        m = mmap.mmap(f.fileno(), 0, prot=mmap.PROT_READ)
    size = len(m)
    buf = np.frombuffer(m, dtype=np.uint8)
    part = -(-size // n)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(part)
    lens = np.minimum(np.uint64(part), np.uint64(size) - offs).astype(np.uint64)
    views = [buf[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]
    variants = {
        "file_auto": lambda: s3.sha256_file_parts(path, offs, lens),
        "file_pread_4k": lambda: s3.sha256_file_parts(path, offs, lens, slice_bytes=4096),
        "file_pread_8k": lambda: s3.sha256_file_parts(path, offs, lens, slice_bytes=8192),
        "file_pread_32k": lambda: s3.sha256_file_parts(path, offs, lens, slice_bytes=32768),
        "caller_mapping": lambda: s3.sha256_batch_host(views),
    }
    ref = None
    times = {k: [] for k in variants}
    for k, f in variants.items():  # warm every variant once (contexts, page cache)
        d = f()
        ref = d if ref is None else ref
        assert np.array_equal(d, ref), k
    for _ in range(reps):
        for k, f in variants.items():
            t0 = time.perf_counter()
            f()
            times[k].append(time.perf_counter() - t0)
    gib = size / 2**30
    for k, t in times.items():
        print(json.dumps({"variant": k, "parts": n, "GiB": round(gib, 3),
                          "median_GiBps": round(gib / float(np.median(t)), 2),
                          "best_GiBps": round(gib / min(t), 2)}), flush=True)


if __name__ == "__main__":
    main()
