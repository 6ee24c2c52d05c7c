#!/usr/bin/env python3
"""Throughput sweep over part counts (not the product): n x 8 MiB parts already in HBM, AUTO
kernel, SHA-256 alone and SHA-256 + MD5; one JSON line per n.  Looks for cliffs -- counts
whose rate falls below the trend (e.g. the partial-last-group one fixed in round 2).

    python tools/sweep_parts.py [--counts 1,7,64,...] [--part-mib 8] > sweep.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = "1,7,64,257,777,1023,1025,1500,1821,2047,2049,2500,3000,4095,4097,5000,6000,8191,8193,12000"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default=DEFAULT)
    ap.add_argument("--part-mib", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    import torch

    import s3client_amd as s3
    from bench import SEED
    counts = [int(x) for x in args.counts.split(",")]
    L = args.part_mib << 20
    nmax = max(counts)
    data = torch.empty(nmax * L, dtype=torch.uint8, device="cuda")
    offs_all = np.arange(nmax, dtype=np.uint64) * np.uint64(L)
    lens_all = np.full(nmax, L, dtype=np.uint64)
    s3.generate_parts(data, offs_all, lens_all, np.arange(nmax, dtype=np.uint64), SEED)
    torch.cuda.synchronize()
    for n in counts:
        offs, lens = offs_all[:n], lens_all[:n]
        with s3.Plan(offs, lens) as plan:
            info = plan.info()
            out = torch.empty((n, 8), dtype=torch.int32, device="cuda")
            plan.launch(data, out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                plan.launch(data, out)
            torch.cuda.synchronize()
            sha_s = (time.perf_counter() - t0) / args.steps
        s3.sha256_md5_batch_device(data, offs, lens)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            s3.sha256_md5_batch_device(data, offs, lens)
        dual_s = (time.perf_counter() - t0) / args.steps
        gib = n * L / 2**30
        print(json.dumps({"parts": n, "part_bytes": L, "kernel": info["kernel"], "grid": info["grid"],
                          "solo": info["solo"], "sha256_ms": round(sha_s * 1e3, 2),
                          "sha256_GiBps": round(gib / sha_s, 2), "dual_ms": round(dual_s * 1e3, 2),
                          "dual_GiBps": round(gib / dual_s, 2)}), flush=True)


if __name__ == "__main__":
    main()
