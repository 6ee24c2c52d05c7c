#!/usr/bin/env python3
"""AUTO routing across the GPU/CPU crossover.

For n in {8, 32, 64, 128, 256, 512, 1024} parts of 8 MiB (C2 parts 0..n-1, generator G), from
pinned host memory (on the device's node) and from pageable memory, time
s3h_sha256_batch_routed with route gpu, cpu, split (the longest parts on the CPU while the
GPU hashes the rest) and auto, round-robin (`--reps` timed calls each after one warm call),
and record the model's estimates and AUTO's choice beside the measured medians.  Every digest
must equal the device-resident run's.  One JSON object on stdout; `auto_over_best` = AUTO's
median / the fastest forced route's (the bar: <= 1.10).

`--dual` (round 6): both upload digests (Content-MD5 + x-amz-content-sha256)
through s3h_sha256_md5_batch_routed, the model's estimates from s3h_route_choose for the dual
digest set; every SHA-256 and MD5 digest vs the device-resident dual run.  The bar: AUTO within
5 % of the fastest forced route for n = 8 ... 1,024.

    python3 tools/route_sweep.py [--reps 3] [--ns 8,32,...] [--dual]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SEED = 20241008
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ns", default="8,32,64,128,256,512,1024")
    ap.add_argument("--sources", default="pinned,pageable", help="of pinned,pageable,file")
    ap.add_argument("--dual", action="store_true", help="both digests (SHA-256 + MD5)")
    a = ap.parse_args()
    import torch

    import s3client_amd as s3
    ns = [int(x) for x in a.ns.split(",")]
    N, L = max(ns), 8 * MIB
    lens = np.full(N, L, dtype=np.uint64)
    offs = np.arange(N, dtype=np.uint64) * np.uint64(L)
    dev = torch.device("cuda", 0)
    data = torch.empty(N * L, dtype=torch.uint8, device=dev)
    s3.generate_parts(data, offs, lens, np.arange(N), SEED)
    if a.dual:
        rs, rm = s3.sha256_md5_batch_device(data, offs, lens)
        ref = (rs.cpu().numpy().view(np.uint32), rm.cpu().numpy().view(np.uint32))
    else:
        ref = s3.sha256_batch_device(data, offs, lens).cpu().numpy().view(np.uint32)
    bufs = {}
    if "pinned" in a.sources:
        pb = s3.PinnedBuffer(N * L, s3.device_numa(0)["node"])
        torch.from_numpy(pb.array).copy_(data)
        bufs["pinned"] = (pb, pb.array)
    if "pageable" in a.sources:
        pg = np.empty(N * L, dtype=np.uint8)
        torch.from_numpy(pg).copy_(data)
        bufs["pageable"] = (None, pg)
    if "file" in a.sources:  # file ranges (page cache): one file of the N parts
        import tempfile
        tmpd = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
        fpath = os.path.join(tmpd, "route_sweep.bin")
        fa = np.empty(N * L, dtype=np.uint8)
        torch.from_numpy(fa).copy_(data)
        fa.tofile(fpath)
        del fa
        bufs["file"] = (fpath, None)
    del data
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    model = s3.route_model()
    rates = s3.route_rates()
    out = {"model": model, "rates": rates, "digests": "sha256+md5" if a.dual else "sha256",
           "model_measure_s": round(time.perf_counter() - t0, 3),
           "part_bytes": L, "reps": a.reps, "cpu_backend": s3.cpu_backend(),
           "host_threads": s3.host_threads(1), "rows": [], "mismatches": 0}
    worst = 0.0
    for src, (handle, arr) in bufs.items():
        for n in ns:
            parts = s3.BufferParts(arr, offs[:n], lens[:n]) if arr is not None else None
            if a.dual:
                ch = s3.route_choose(lens[:n], s3.route_rates(), "both", source=src)
                est_route, g_est, c_est = ch["route"], ch["gpu_s"], ch["cpu_s"]
                k_est, tg_est, s_est = ch["cpu_parts"], ch["stage_threads"], ch["split_s"]
            else:
                ch = s3.route_choose(lens[:n], s3.route_rates(), "sha256", source=src)
                est_route, g_est, c_est = ch["route"], ch["gpu_s"], ch["cpu_s"]
                k_est, tg_est, s_est = ch["cpu_parts"], ch["stage_threads"], ch["split_s"]
            times = {r: [] for r in ("gpu", "cpu", "split", "auto")}
            taken = None
            for k in range(a.reps + 1):
                for r in times:
                    t1 = time.perf_counter()
                    if src == "file" and a.dual:
                        ds, dm, tk = s3.sha256_md5_file_parts_routed(handle, offs[:n], lens[:n], ndevices=1, route=r)
                    elif src == "file":
                        d, tk = s3.sha256_file_parts_routed(handle, offs[:n], lens[:n], ndevices=1, route=r)
                    elif a.dual:
                        ds, dm, tk = s3.sha256_md5_batch_routed(parts, ndevices=1, route=r)
                    else:
                        d, tk = s3.sha256_batch_routed(parts, ndevices=1, route=r)
                    dt = time.perf_counter() - t1
                    if k:
                        times[r].append(dt)
                    if r == "auto":
                        taken = tk
                    ok = (np.array_equal(ds, ref[0][:n]) and np.array_equal(dm, ref[1][:n])) if a.dual \
                        else np.array_equal(d, ref[:n])
                    out["mismatches"] += int(not ok)
            med = {r: float(np.median(v)) for r, v in times.items()}
            ratio = med["auto"] / min(med["gpu"], med["cpu"], med["split"])
            worst = max(worst, ratio)
            out["rows"].append({
                "source": src, "n": n, "GiB": round(n * L / 2**30, 3),
                "median_s": {r: round(v, 4) for r, v in med.items()},
                "all_s": {r: [round(x, 4) for x in v] for r, v in times.items()},
                "GiBps": {r: round(n * L / 2**30 / v, 2) for r, v in med.items()},
                "auto_taken": taken, "faster": min(("gpu", "cpu", "split"), key=lambda r: med[r]),
                "auto_over_best": round(ratio, 4),
                "model": {"route": est_route, "gpu_s": round(g_est, 4), "cpu_s": round(c_est, 4),
                          "split_s": round(s_est, 4), "split_cpu_parts": k_est,
                          "split_stage_threads": tg_est}})
            print(f"[route_sweep] {src} n={n}: gpu {med['gpu']:.4f} cpu {med['cpu']:.4f} split {med['split']:.4f} "
                  f"auto {med['auto']:.4f} ({taken}) model gpu {g_est:.4f} cpu {c_est:.4f} split {s_est:.4f} ({k_est})",
                  file=sys.stderr, flush=True)
    if "file" in bufs:
        os.remove(bufs["file"][0])
    out["worst_auto_over_best"] = round(worst, 4)
    out["rates_after"] = s3.route_rates()
    print(json.dumps(out))
    return 0 if out["mismatches"] == 0 else 3


if __name__ == "__main__":
    sys.exit(main())
