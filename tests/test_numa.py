"""NUMA placement of the host path (CPU).

The library reads a device's node from sysfs -- <root>/bus/pci/devices/<bdf>/numa_node and
local_cpulist, S3H_SYSFS_ROOT replacing /sys -- and binds each device's pinned staging and
copy threads there (capi.hip "NUMA placement").  These tests build fake sysfs trees shaped
like the GPU box's (profiles/r05_numa_probe.json: two nodes, GPUs on node 1 with CPUs
64-127,192-255) and check the bus ID -> node -> CPU list mapping, the affinity intersection,
the policy switch and the page-node query, none of which needs a GPU.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import s3client_amd as s3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fake_sysfs(tmp_path, devices: dict, nodes: dict | None = None) -> str:
    """devices: {bdf: (numa_node text, local_cpulist text or None)}; nodes: {k: cpulist}."""
    root = tmp_path / "sys"
    for bdf, (node, cpus) in devices.items():
        d = root / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text(node + "\n")
        if cpus is not None:
            (d / "local_cpulist").write_text(cpus + "\n")
    for k, cpus in (nodes or {}).items():
        d = root / "devices" / "system" / "node" / f"node{k}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
    return str(root)


def run_child(code: str, env: dict) -> str:
    r = subprocess.run([sys.executable, "-c", code], env={**os.environ, **env}, cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


def test_bus_id_maps_to_node_and_cpulist(tmp_path, monkeypatch):
    ncpu = max(os.sched_getaffinity(0)) + 1
    root = fake_sysfs(tmp_path, {
        "0000:f1:00.0": ("1", f"{ncpu // 2}-{ncpu - 1}"),   # GPU behind socket 1
        "0000:05:00.0": ("0", f"0-{ncpu // 2 - 1}"),        # GPU behind socket 0
        "0000:11:00.0": ("-1", ""),                          # no NUMA information
    })
    monkeypatch.setenv("S3H_SYSFS_ROOT", root)
    mine = os.sched_getaffinity(0)
    r1 = s3.pci_numa("0000:F1:00.0")  # upper case as some tools print it
    assert r1["node"] == 1 and r1["local_cpulist"] == f"{ncpu // 2}-{ncpu - 1}"
    assert r1["usable_cpus"] == len([c for c in mine if c >= ncpu // 2])
    r0 = s3.pci_numa("0000:05:00.0")
    assert r0["node"] == 0 and r0["usable_cpus"] == len([c for c in mine if c < ncpu // 2])
    rn = s3.pci_numa("0000:11:00.0")
    assert rn["node"] == -1 and rn["usable_cpus"] == 0
    with pytest.raises(s3.S3HashError, match="cannot read"):
        s3.pci_numa("0000:99:00.0")


def test_cpulist_forms(tmp_path, monkeypatch):
    lists = {"0000:01:00.0": "0,2-3,5", "0000:02:00.0": "3", "0000:03:00.0": "0-1,x"}
    root = fake_sysfs(tmp_path, {b: ("0", c) for b, c in lists.items()})
    monkeypatch.setenv("S3H_SYSFS_ROOT", root)
    mine = os.sched_getaffinity(0)
    assert s3.pci_numa("0000:01:00.0")["usable_cpus"] == len(mine & {0, 2, 3, 5})
    assert s3.pci_numa("0000:02:00.0")["usable_cpus"] == len(mine & {3})
    assert s3.pci_numa("0000:03:00.0")["usable_cpus"] == 0  # malformed: never bind


def test_usable_cpus_follow_a_narrowed_affinity(tmp_path):
    """A process pinned to two CPUs may only bind its copy threads within them."""
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 3:
        pytest.skip("needs 3 CPUs")
    root = fake_sysfs(tmp_path, {"0000:f1:00.0": ("1", f"{cpus[1]}-{cpus[-1]}")})
    code = (f"import os;os.sched_setaffinity(0,{cpus[:2]!r});import s3client_amd as s3;"
            "print(s3.pci_numa('0000:f1:00.0')['usable_cpus'])")
    assert run_child(code, {"S3H_SYSFS_ROOT": root}) == "1"  # only cpus[1] is both


def test_policy_switch_and_env():
    prev = s3.host_numa("off")
    try:
        assert s3.host_numa(1) == -2
        assert s3.host_numa("local") == 1
        with pytest.raises(s3.S3HashError):
            s3.host_numa(-3)
    finally:
        s3.host_numa(prev)
    code = "import s3client_amd as s3;print(s3.host_numa('local'))"
    assert run_child(code, {"S3H_HOST_NUMA": "off"}) == "-2"
    assert run_child(code, {"S3H_HOST_NUMA": "0"}) == "0"
    assert run_child(code, {"S3H_HOST_NUMA": "local"}) == "-1"


def test_mem_node_of_host_pages():
    a = np.ones(1 << 20, dtype=np.uint8)
    node = s3.mem_node(a)
    with open("/proc/self/status") as f:
        mems = next(l.split(":")[1].strip() for l in f if l.startswith("Mems_allowed_list"))
    allowed = set()
    for part in mems.split(","):
        lo, _, hi = part.partition("-")
        allowed |= set(range(int(lo), int(hi or lo) + 1))
    assert node in allowed


def test_numa_symbols_declared_and_exported():
    hdr = open(os.path.join(ROOT, "include", "s3hash.h")).read()
    for sym in ("s3h_pci_numa", "s3h_device_numa_node", "s3h_host_numa", "s3h_host_numa_info",
                "s3h_host_alloc", "s3h_host_free", "s3h_mem_node"):
        assert f" {sym}(" in hdr, sym
        assert hasattr(s3._native.lib(), sym)
