#!/usr/bin/env python3
"""NUMA layout of the GPU box as this process sees it (first step).

Prints one JSON object: every AMD GPU's PCI function with its sysfs numa_node and
local_cpulist, the host's nodes (cpulist, free memory), this process's allowed CPUs and
memory nodes (/proc/self/status), the cgroup cpuset/quota, and -- with --h2d -- the pinned
H2D rate of an 8 GiB-bounded buffer whose pages were bound (mbind) to each allowed node,
registered with hipHostRegister and copied to device 0, timed with HIP events.

    python3 tools/numa_probe.py [--h2d] [--mib 1024]
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import mmap
import os
import time


def read(path: str, default: str = "") -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def gpus() -> list:
    out = []
    for d in sorted(glob.glob("/sys/bus/pci/devices/*")):
        if read(d + "/vendor") != "0x1002":
            continue
        cls = read(d + "/class")
        if not (cls.startswith("0x0380") or cls.startswith("0x0300") or cls.startswith("0x1200")):
            continue
        out.append({"bdf": os.path.basename(d), "class": cls, "device": read(d + "/device"),
                    "numa_node": read(d + "/numa_node"), "local_cpulist": read(d + "/local_cpulist")})
    return out


def nodes() -> list:
    out = []
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        mem = {l.split(":")[0].split()[-1]: l.split(":")[1].strip()
               for l in read(d + "/meminfo").splitlines() if ":" in l}
        out.append({"node": os.path.basename(d), "cpulist": read(d + "/cpulist"),
                    "MemTotal": mem.get("MemTotal"), "MemFree": mem.get("MemFree")})
    return out


def status() -> dict:
    s = {}
    for l in read("/proc/self/status").splitlines():
        k = l.split(":")[0]
        if k in ("Cpus_allowed_list", "Mems_allowed_list"):
            s[k] = l.split(":", 1)[1].strip()
    return s


def cgroup() -> dict:
    c = {}
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective",
              "/sys/fs/cgroup/cpuset.mems.effective", "/sys/fs/cgroup/cpuset/cpuset.cpus",
              "/sys/fs/cgroup/cpuset/cpuset.mems", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us",
              "/proc/self/cgroup"):
        v = read(p, None)
        if v is not None:
            c[p] = v[:400]
    return c


def parse_list(s: str) -> list:
    out = []
    for part in s.split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


MPOL_BIND = 2
SYS_mbind = 237  # x86_64
SYS_get_mempolicy = 239
MPOL_F_NODE, MPOL_F_ADDR = 1, 2


def h2d_by_node(mib: int) -> list:
    libc = ctypes.CDLL(None, use_errno=True)
    hip = ctypes.CDLL("libamdhip64.so")
    size = mib << 20
    res = []
    dptr = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(size)) == 0
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    hip.hipEventCreate(ctypes.byref(e0))
    hip.hipEventCreate(ctypes.byref(e1))
    allowed = parse_list(status().get("Mems_allowed_list", "0"))
    for node in allowed:
        m = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        addr = ctypes.addressof(ctypes.c_char.from_buffer(m))
        mask = ctypes.c_ulong(1 << node) if node < 64 else None
        rc = libc.syscall(SYS_mbind, ctypes.c_void_p(addr), ctypes.c_ulong(size), MPOL_BIND,
                          ctypes.byref(mask), ctypes.c_ulong(65), 0)
        err = ctypes.get_errno() if rc else 0
        m.write(b"\x5a" * size)  # first touch
        got = ctypes.c_int(-1)
        libc.syscall(SYS_get_mempolicy, ctypes.byref(got), None, 0, ctypes.c_void_p(addr),
                     MPOL_F_NODE | MPOL_F_ADDR)
        r = {"bound_node": node, "mbind_rc": rc, "errno": err, "page0_node": got.value}
        t0 = time.perf_counter()
        reg = hip.hipHostRegister(ctypes.c_void_p(addr), ctypes.c_size_t(size), 0)
        r["register_s"] = round(time.perf_counter() - t0, 3)
        r["register_rc"] = reg
        if reg == 0:
            best = 1e9
            for _ in range(4):
                hip.hipEventRecord(e0, None)
                hip.hipMemcpyAsync(dptr, ctypes.c_void_p(addr), ctypes.c_size_t(size), 1, None)
                hip.hipEventRecord(e1, None)
                hip.hipEventSynchronize(e1)
                ms = ctypes.c_float()
                hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1)
                best = min(best, ms.value)
            r["h2d_GiBps"] = round(size / 2**30 / (best / 1e3), 2)
            hip.hipHostUnregister(ctypes.c_void_p(addr))
        res.append(r)
        del addr
        m.close()
    # hipHostMalloc default: where do its pages land?
    hp = ctypes.c_void_p()
    if hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(size), 0) == 0:
        ctypes.memset(hp, 0x5a, size)
        got = ctypes.c_int(-1)
        libc.syscall(SYS_get_mempolicy, ctypes.byref(got), None, 0, hp, MPOL_F_NODE | MPOL_F_ADDR)
        best = 1e9
        for _ in range(4):
            hip.hipEventRecord(e0, None)
            hip.hipMemcpyAsync(dptr, hp, ctypes.c_size_t(size), 1, None)
            hip.hipEventRecord(e1, None)
            hip.hipEventSynchronize(e1)
            ms = ctypes.c_float()
            hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1)
            best = min(best, ms.value)
        res.append({"hipHostMalloc_default_page0_node": got.value,
                    "h2d_GiBps": round(size / 2**30 / (best / 1e3), 2),
                    "caller_cpu": os.sched_getaffinity(0).__len__()})
        hip.hipHostFree(hp)
    hip.hipFree(dptr)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h2d", action="store_true")
    ap.add_argument("--mib", type=int, default=1024)
    a = ap.parse_args()
    out = {"gpus": gpus(), "nodes": nodes(), "self": status(), "cgroup": cgroup(),
           "cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
           "env": {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                  "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")}}
    if a.h2d:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        hip.hipDeviceGetPCIBusId(buf, 64, 0)
        out["hip_device0_bdf"] = buf.value.decode().lower()
        out["h2d_by_node"] = h2d_by_node(a.mib)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
