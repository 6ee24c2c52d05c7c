#!/usr/bin/env python3
"""Local/remote NUMA A/B of the host path on a dual-socket GPU box.

The same C2 parts (generator G, parts 0..n-1 of 8 MiB) are placed in host memory on the
device's node ("local") and on the other node ("remote"), as pageable memory (the path then
stages through the pinned ring with host copy threads) and as pinned memory (direct DMA), and
hashed by s3h_sha256_batch_host under three placement policies for the library's staging
ring and copy threads: local (the default), remote (s3h_host_numa(<other node>)), off (the
runtime's placement, unbound threads).  Every combination runs `--reps` times, round-robin,
and every digest must equal the device-resident run's.  With --load T the whole A/B runs a
second time while T background threads, bound to the device node's CPUs, copy a buffer on the
remote node into one on the device's node (numpy copyto, 256 MiB at a time): the inter-socket
traffic that the other GPUs of an 8-GPU node reading remote memory would add.  One JSON
object on stdout.

    python3 tools/numa_ab.py [--parts 1024] [--reps 5] [--load 8]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import mmap
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEED = 20241008
MIB = 1 << 20
SYS_mbind = 237  # x86_64
MPOL_BIND = 2


def pageable_on(nbytes: int, node: int):
    """Anonymous pageable memory whose pages are bound to `node` (mbind), as a numpy array."""
    m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    arr = np.frombuffer(m, dtype=np.uint8)
    mask = ctypes.c_ulong(1 << node)
    libc = ctypes.CDLL(None, use_errno=True)
    rc = libc.syscall(SYS_mbind, ctypes.c_void_p(arr.ctypes.data), ctypes.c_ulong(nbytes),
                      MPOL_BIND, ctypes.byref(mask), ctypes.c_ulong(65), 0)
    if rc != 0:
        raise OSError(ctypes.get_errno(), f"mbind to node {node}")
    return m, arr


def _cpulist(s: str) -> list:
    out = []
    for part in s.split(","):
        if part:
            lo, _, hi = part.partition("-")
            out += list(range(int(lo), int(hi or lo) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--load", type=int, default=0)
    a = ap.parse_args()
    import torch

    import bench
    import s3client_amd as s3
    dev = torch.device("cuda", 0)
    n, L = a.parts, 8 * MIB
    lens = np.full(n, L, dtype=np.uint64)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    data = torch.empty(n * L, dtype=torch.uint8, device=dev)
    s3.generate_parts(data, offs, lens, np.arange(n), SEED)
    ref = s3.sha256_batch_device(data, offs, lens).cpu().numpy().view(np.uint32)
    dn = s3.device_numa(0)["node"]
    others = [k for k in bench.allowed_mem_nodes() if k != dn]
    if dn < 0 or not others:
        print(json.dumps({"error": f"needs a multi-node host (device node {dn}, "
                                   f"allowed {bench.allowed_mem_nodes()})"}))
        return 1
    rn = others[0]
    sources = {}
    for side, node in (("local", dn), ("remote", rn)):
        m, arr = pageable_on(n * L, node)
        torch.from_numpy(arr).copy_(data)
        sources[f"pageable_{side}"] = (m, arr)
        pb = s3.PinnedBuffer(n * L, node)
        torch.from_numpy(pb.array).copy_(data)
        sources[f"pinned_{side}"] = (pb, pb.array)
    del data
    torch.cuda.empty_cache()
    policies = {"local": "local", "remote": rn, "off": "off"}
    gib = n * L / 2**30
    res = {"device": s3.device_pci_bus_id(0), "device_node": dn, "remote_node": rn,
           "parts": n, "part_bytes": L, "reps": a.reps,
           "source_nodes": {k: s3.mem_node(v[1]) for k, v in sources.items()},
           "runs": {}, "mismatches": 0}
    combos = [(src, pol) for src in sources for pol in policies
              if src.startswith("pageable") or pol == "local"]  # pinned parts never stage
    parts = {src: s3.BufferParts(v[1], offs, lens) for src, v in sources.items()}

    def ab(tag):
        times = {c: [] for c in combos}
        placed = {}
        for _ in range(a.reps):
            for pol in policies:
                s3.host_numa(policies[pol])  # a change re-places the context: warm it untimed
                s3.sha256_batch_host(parts["pageable_local"], ndevices=1)
                for src in sources:
                    if (src, pol) not in times:
                        continue
                    t0 = time.perf_counter()
                    out = s3.sha256_batch_host(parts[src], ndevices=1)
                    times[(src, pol)].append(time.perf_counter() - t0)
                    placed.setdefault((src, pol), s3.host_numa_info(0))
                    res["mismatches"] += int(not np.array_equal(out, ref))
        s3.host_numa("local")
        res[tag] = {}
        for (src, pol), ts in times.items():
            res[tag][f"{src}/staging_{pol}"] = {
                "GiBps_median": round(gib / float(np.median(ts)), 3),
                "GiBps": [round(gib / t, 2) for t in ts], "placement": placed[(src, pol)]}

    ab("runs")
    if a.load:
        import threading
        chunk = 256 * MIB
        _, far = pageable_on(4 * chunk, rn)
        _, near = pageable_on(4 * chunk, dn)
        far[:] = 1
        near[:] = 0
        cpus = sorted(set(range(os.cpu_count())) & os.sched_getaffinity(0))
        local_cpus = [c for c in cpus if c in set(
            _cpulist(s3.device_numa(0)["local_cpulist"]))] or cpus
        stop = threading.Event()
        moved = [0] * a.load

        def loader(k):
            os.sched_setaffinity(0, {local_cpus[k % len(local_cpus)]})
            i = 0
            while not stop.is_set():
                o = (i % 4) * chunk
                np.copyto(near[o:o + chunk], far[o:o + chunk])
                moved[k] += chunk
                i += 1
        th = [threading.Thread(target=loader, args=(k,), daemon=True) for k in range(a.load)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        ab("runs_under_load")
        stop.set()
        for t in th:
            t.join()
        res["load"] = {"threads": a.load, "direction": f"node {rn} -> node {dn} memcpy",
                       "GBps": round(sum(moved) / (time.perf_counter() - t0) / 1e9, 2)}
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
