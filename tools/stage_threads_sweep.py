#!/usr/bin/env python3
"""GPU host path from staged sources with the staging threads per device capped
(S3H_STAGE_THREADS = 2 ... 16): C2's 1,024 x 8 MiB parts from pageable memory and from a file in
the page cache, median of --reps calls after a warm one, digests vs the first call.  One JSON
object.

    python3 tools/stage_threads_sweep.py [--ts 2,4,6,8,12,16] [--reps 3]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ts", default="2,4,6,8,12,16")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    import s3client_amd as s3
    n, L = 1024, 8 * MIB
    lens = np.full(n, L, dtype=np.uint64)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    dev = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    s3.generate_parts(dev, offs, lens, np.arange(n), 20241008)
    host = dev.cpu().numpy()
    del dev
    torch.cuda.empty_cache()
    res = {"rows": [], "mismatches": 0, "host_threads": s3.host_threads(1)}
    ref = None
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        path = os.path.join(td, "c2.bin")
        host.tofile(path)
        parts = s3.BufferParts(host, offs, lens)
        for source in ("pageable", "file"):
            for t in [int(x) for x in a.ts.split(",")]:
                os.environ["S3H_STAGE_THREADS"] = str(t)
                fn = (lambda: s3.sha256_batch_host(parts, ndevices=1)) if source == "pageable" else \
                     (lambda: s3.sha256_file_parts(path, offs, lens, ndevices=1))
                d = fn()
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    d = fn()
                    ts.append(time.perf_counter() - t0)
                ref = d if ref is None else ref
                res["mismatches"] += int(not np.array_equal(d, ref))
                row = {"source": source, "stage_threads": t,
                       "GiBps": round(n * L / 2**30 / float(np.median(ts)), 2)}
                res["rows"].append(row)
                print(json.dumps(row), file=sys.stderr, flush=True)
    os.environ.pop("S3H_STAGE_THREADS", None)
    print(json.dumps(res))
    return 1 if res["mismatches"] else 0


if __name__ == "__main__":
    sys.exit(main())
