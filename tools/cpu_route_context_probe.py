#!/usr/bin/env python3
"""Why the CPU route runs ~2x slower inside tools/route_sweep.py than its own model and than
tools/cpu_dual_probe (same cpu_batch, same 8 MiB parts) on the GPU box.

Times s3h_sha256_md5_batch_routed(route="cpu") over 64 x 8 MiB parts in successive process
states -- before any HIP initialisation, torch + HIP initialised, after GPU-route calls, from a
pinned buffer -- and beside each the process's CPU time (user+sys over wall = the parallelism
the threads actually got) and the cgroup's throttling counters (cpu.stat nr_throttled /
throttled_usec).  One JSON object on stdout.

    python3 tools/cpu_route_context_probe.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MIB = 1 << 20


def cgroup_stat() -> dict:
    out = {}
    for p in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat"):
        try:
            for line in open(p):
                k, v = line.split()
                out[k] = int(v)
            break
        except OSError:
            continue
    return out


def cgroup_max() -> str:
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            return open(p).read().strip()
        except OSError:
            pass
    return ""


def timed(fn, reps: int = 3) -> dict:
    fn()  # warm
    runs = []
    for _ in range(reps):
        c0, t0, s0 = os.times(), time.perf_counter(), cgroup_stat()
        fn()
        wall = time.perf_counter() - t0
        c1, s1 = os.times(), cgroup_stat()
        cpu = (c1.user - c0.user) + (c1.system - c0.system)
        runs.append({"wall_s": round(wall, 4), "cpu_s": round(cpu, 3),
                     "parallelism": round(cpu / wall, 2),
                     "throttled": {k: s1.get(k, 0) - s0.get(k, 0)
                                   for k in ("nr_throttled", "throttled_usec") if k in s1}})
    best = min(r["wall_s"] for r in runs)
    return {"best_wall_s": best, "runs": runs}


def main():
    import s3client_amd as s3
    n, L = 64, 8 * MIB
    rng = np.random.default_rng(5)
    big = rng.integers(0, 256, n * L, dtype=np.uint8)
    parts = [big[i * L:(i + 1) * L] for i in range(n)]
    gib = n * L / 2**30
    res = {"parts": n, "part_bytes": L, "affinity_cpus": len(os.sched_getaffinity(0)),
           "cgroup_cpu_max": cgroup_max(), "host_plan": s3.host_plan([None]), "phases": {}}

    def cpu_dual():
        s3.sha256_md5_batch_routed(parts, route="cpu")

    def cpu_sha():
        s3.sha256_batch_routed(parts, route="cpu")

    def phase(name):
        d = timed(cpu_dual)
        s = timed(cpu_sha)
        res["phases"][name] = {"dual": d, "sha256": s,
                               "dual_GiBps": round(gib / d["best_wall_s"], 2),
                               "sha256_GiBps": round(gib / s["best_wall_s"], 2)}
        print(f"[ctx] {name}: dual {gib / d['best_wall_s']:.2f} GiB/s "
              f"(par {d['runs'][-1]['parallelism']}), sha256 {gib / s['best_wall_s']:.2f} GiB/s",
              file=sys.stderr, flush=True)

    phase("before_hip_init")
    import torch
    torch.cuda.init()
    dev_buf = torch.empty(64 * MIB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    phase("torch_hip_initialised")
    for _ in range(3):
        s3.sha256_md5_batch_routed(parts, route="gpu")
    phase("after_gpu_route_calls")
    rates = s3.route_rates()
    res["route_rates"] = {k: rates[k] for k in ("cpu_threads", "cpu_bytes_per_s",
                                                "cpu_all_bytes_per_s") if k in rates}
    pb = s3.PinnedBuffer(n * L, s3.device_numa(0)["node"])
    pb.array[:] = big
    parts[:] = [pb.array[i * L:(i + 1) * L] for i in range(n)]
    phase("pinned_source")
    del dev_buf
    print(json.dumps(res))


if __name__ == "__main__":
    main()
