#!/usr/bin/env python3
"""Where the route model's GPU estimate misses (round 6, from the S3H_TRACE_ROUTE log of
tests/test_gpu_route_adapt.py): the split's GPU side on a ragged set (300 parts of U[1, 16]
MiB) ran ~3x its estimate, and on C2 file ranges with 5-8 staging threads ~1.5x.

Times the GPU route alone (s3h_*_batch_routed route="gpu", 3 reps, best) beside the model's
raw GPU estimate (s3h_route_choose with the corrections at 1):
  * the ragged set and its split GPU side (the set minus its 136 longest parts), pinned and
    pageable, SHA-256 / both digests;
  * C2 (1,024 x 8 MiB) from a file with S3H_STAGE_THREADS = 5, 8, 16, both digests.
One JSON object on stdout.

    python3 tools/route_gpu_side_probe.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MIB = 1 << 20
SEED = 20241008


def gen(torch, s3, lens):
    lens = np.asarray(lens, dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum((lens + 255) // 256 * 256)[:-1]]).astype(np.uint64)
    dev = torch.empty(int(offs[-1] + lens[-1]) + 256, dtype=torch.uint8, device="cuda")
    s3.generate_parts(dev, offs, lens, np.arange(lens.size), SEED)
    host = dev.cpu().numpy()
    del dev
    torch.cuda.empty_cache()
    return host, offs, lens


def best(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(min(ts), 4), [round(t, 4) for t in ts]


def main():
    import torch
    import s3client_amd as s3
    out = {"rows": []}
    R0 = dict(s3.route_rates(), gpu_factor=[1.0] * 3, cpu_factor=[1.0] * 3)
    out["rates"] = {k: R0[k] for k in ("chain_bytes_per_s", "h2d_bytes_per_s", "staged_bytes_per_s",
                                       "call_s", "cpu_threads")}
    rng = np.random.default_rng(606)
    lens = rng.integers(1 * MIB, 16 * MIB, 300)
    lens[:4] = [0, 1, 55, 64]
    host, offs, lens = gen(torch, s3, lens)
    order = np.argsort(-lens.astype(np.int64), kind="stable")
    sets = {"ragged300": np.arange(lens.size), "ragged300_gpu_side": np.sort(order[136:])}
    for source in ("pinned", "pageable"):
        buf = torch.empty(host.size, dtype=torch.uint8, pin_memory=source == "pinned")
        buf.numpy()[:] = host
        h = buf.numpy()
        for name, idx in sets.items():
            views = [h[int(offs[i]):int(offs[i]) + int(lens[i])] for i in idx]
            L = lens[idx]
            for dig, fn in (("sha256", lambda: s3.sha256_batch_routed(views, route="gpu")),
                            ("both", lambda: s3.sha256_md5_batch_routed(views, route="gpu"))):
                t, ts = best(fn)
                est = s3.route_choose(L, R0, dig, source=source)["gpu_s"]
                row = {"set": name, "source": source, "digests": dig, "n": int(L.size),
                       "longest_MiB": round(float(L.max()) / MIB, 2), "GiB": round(float(L.sum()) / 2**30, 3),
                       "gpu_s": t, "all_s": ts, "model_gpu_s": round(est, 4), "ratio": round(t / est, 3)}
                out["rows"].append(row)
                print(f"[probe] {row}", file=sys.stderr, flush=True)
        del buf
    # C2 from a file, staging-thread caps
    host, offs, lens = gen(torch, s3, np.full(1024, 8 * MIB))
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        path = os.path.join(d, "c2.bin")
        host.tofile(path)
        for tg in (5, 8, 16):
            os.environ["S3H_STAGE_THREADS"] = str(tg)
            t, ts = best(lambda: s3.sha256_md5_file_parts_routed(path, offs, lens, route="gpu"))
            R = dict(R0, cpu_threads=R0["cpu_threads"])
            est = s3.route_choose(lens, R, "both", source="file")["gpu_s"]
            row = {"set": "c2_file", "stage_threads": tg, "digests": "both", "gpu_s": t, "all_s": ts,
                   "model_gpu_s_all_threads": round(est, 4)}
            out["rows"].append(row)
            print(f"[probe] {row}", file=sys.stderr, flush=True)
        os.environ.pop("S3H_STAGE_THREADS", None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
