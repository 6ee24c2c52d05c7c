#!/usr/bin/env python3
"""The split route on staged sources: C2's 1,024 x 8 MiB parts from pageable memory and from a
file in the page cache, the GPU side's staging threads per device fixed at each --tgs value
(S3H_SPLIT_STAGE_THREADS; the CPU side gets the other host threads) and then left to the model;
the forced GPU and CPU routes beside them.  Median of --reps calls after a warm one, the
model's estimate and CPU share for each, digests vs the first GPU result.  One JSON object.

    python3 tools/split_stage_sweep.py [--tgs 2,4,6,8,10,12] [--reps 3]
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
    ap.add_argument("--tgs", default="2,4,6,8,10,12")
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
    host = dev.cpu().numpy()
    del dev
    torch.cuda.empty_cache()
    gib = n * L / 2**30
    model = s3.route_model()
    res = {"parts": n, "part_bytes": L, "reps": a.reps, "model": model, "rows": [], "mismatches": 0}
    ref = None
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        path = os.path.join(td, "c2.bin")
        host.tofile(path)
        for source in ("pageable", "file"):
            parts = s3.BufferParts(host, offs, lens)

            def call(route):
                if source == "file":
                    return s3.sha256_file_parts_routed(path, offs, lens, ndevices=1, route=route)
                return s3.sha256_batch_routed(parts, ndevices=1, route=route)

            for tg in ["gpu", "cpu"] + [int(x) for x in a.tgs.split(",")] + ["model"]:
                route = tg if tg in ("gpu", "cpu") else "split"
                if isinstance(tg, int):
                    os.environ["S3H_SPLIT_STAGE_THREADS"] = str(tg)
                else:
                    os.environ.pop("S3H_SPLIT_STAGE_THREADS", None)
                est = s3.route_split_estimate(lens, model, ndevices=1, source=source) if route == "split" else None
                d, taken = call(route)
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    d, taken = call(route)
                    ts.append(time.perf_counter() - t0)
                if ref is None:
                    ref = d
                res["mismatches"] += int(not np.array_equal(d, ref))
                t = float(np.median(ts))
                row = {"source": source, "route": route, "stage_threads": tg, "taken": taken,
                       "s": round(t, 4), "GiBps": round(gib / t, 2)}
                if est:
                    row["model"] = {"cpu_parts": est[0], "stage_threads": est[1], "s": round(est[2], 4)}
                res["rows"].append(row)
                print(json.dumps(row), file=sys.stderr, flush=True)
        os.environ.pop("S3H_SPLIT_STAGE_THREADS", None)
    print(json.dumps(res))
    return 1 if res["mismatches"] else 0


if __name__ == "__main__":
    sys.exit(main())
