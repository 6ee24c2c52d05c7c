#!/usr/bin/env python3
"""Calibrate the CPU baseline restatement (oracle/cpu_baseline.c) against the REAL lib/hash.

Build container only (needs /root/reference).  Both are compiled here with the reference's
release flags `-Ofast -march=native -flto` (lib/CMakeLists.txt:45) into oracle/_ref/, then
timed alternately on the same parts (generator G, 8 MiB, plus a 4 KiB-scratch-sized set) with
1 thread.  Writes profiles/r02_cpu_baseline_calibration.json: ratio = restatement GiB/s /
lib/hash GiB/s (target ~1.0), and checks both produce identical digests.

    python tools/calibrate_cpu_baseline.py
"""
import ctypes
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(ROOT, "oracle", "_ref")
FLAGS = ["-Ofast", "-march=native", "-flto", "-DNDEBUG", "-fPIC", "-shared", "-pthread"]
u64p = ctypes.POINTER(ctypes.c_uint64)


def build():
    os.makedirs(OUT, exist_ok=True)
    ref_so = os.path.join(OUT, "libref_hash_native.so")
    base_so = os.path.join(OUT, "libcpubase_native.so")
    hash_dir = os.path.join(REF, "lib", "hash")
    subprocess.run(["g++", "-std=c++17", *FLAGS, "-I" + hash_dir, "-o", ref_so,
                    os.path.join(ROOT, "oracle", "ref_wrap.cpp")] +
                   [os.path.join(hash_dir, f) for f in ("sha256.cpp", "hmac256.cpp", "utility.cpp", "md5.cpp")],
                   check=True)
    subprocess.run(["gcc", "-std=gnu11", *FLAGS, "-o", base_so,
                    os.path.join(ROOT, "oracle", "cpu_baseline.c")], check=True)
    return ref_so, base_so


def main():
    ref_so, base_so = build()
    ref = ctypes.CDLL(ref_so).ref_sha256_batch
    base = ctypes.CDLL(base_so).base_sha256_batch
    for f in (ref, base):
        f.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    sys.path.insert(0, ROOT)
    from tests.oracle_lib import Oracle
    orc = Oracle()
    results = {}
    for name, L, n in (("8MiB", 8 << 20, 12), ("3000B", 3000, 40000)):
        buf = np.concatenate([np.frombuffer(orc.generate(p, L), np.uint8) for p in range(min(n, 64))])
        reps = (n + 63) // 64
        buf = np.tile(buf, reps)[: n * L] if reps > 1 else buf
        offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
        lens = np.full(n, L, dtype=np.uint64)
        outs, times = {}, {"lib/hash": [], "restatement": []}
        for rep in range(5):
            for k, fn in (("lib/hash", ref), ("restatement", base)):
                o = np.zeros((n, 8), np.uint32)
                t0 = time.perf_counter()
                fn(buf.ctypes.data, offs.ctypes.data_as(u64p), lens.ctypes.data_as(u64p), n, o.ctypes.data, 1)
                times[k].append(time.perf_counter() - t0)
                outs[k] = o
        assert np.array_equal(outs["lib/hash"], outs["restatement"]), name
        gib = n * L / 2**30
        r = {k: round(gib / min(v), 4) for k, v in times.items()}
        results[name] = {"parts": n, "part_bytes": L, "GiBps_best_of_5": r,
                         "ratio_restatement_over_libhash": round(r["restatement"] / r["lib/hash"], 4),
                         "digests_identical": True}
    cpu = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "")
    doc = {"what": "oracle/cpu_baseline.c vs the real lib/hash (reference lib/hash/*.cpp), both built "
                   "-Ofast -march=native -flto here, 1 thread, best of 5 alternating runs",
           "host": {"cpu_model": cpu, "machine": platform.machine()}, "results": results}
    path = os.path.join(ROOT, "profiles", "r02_cpu_baseline_calibration.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
