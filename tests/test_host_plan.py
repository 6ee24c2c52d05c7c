"""The host path's thread plan on an 8-GPU, two-socket node, checked before the driver runs it
(CPU).

s3h_host_plan applies the rules the host pipeline and the split route run by -- staging threads
per device min(16, max(1, cpus / N)), each device's threads bound to its NUMA node's CPUs
within the affinity, the split route's CPU side every thread (pinned parts) or what the
per-device staging shares leave (staged sources) -- over a fake sysfs tree shaped like an
MI355X node (two sockets, GPUs 0-3 behind node 0 with CPUs 0-63,128-191, GPUs 4-7 behind node 1
with CPUs 64-127,192-255) and fake cgroup quotas of 16, 64 and 256 CPUs, for N = 1, 2, 4, 8
devices.  The reference's jobs run wherever the host schedules them (lib/src/upload.cpp:136-140).
"""
import os

import pytest

import s3client_amd as s3

NODE_CPUS = {0: "0-63,128-191", 1: "64-127,192-255"}
BDFS = ["0000:0a:00.0", "0000:23:00.0", "0000:5a:00.0", "0000:72:00.0",  # the GPU box (r05_numa_probe.json)
        "0000:8b:00.0", "0000:a4:00.0", "0000:d9:00.0", "0000:f1:00.0"]


def fake_node(tmp_path, quota_line: str | None = None, v1: tuple | None = None) -> str:
    root = tmp_path / "sys"
    for k, bdf in enumerate(BDFS):
        d = root / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        node = 0 if k < 4 else 1
        (d / "numa_node").write_text(f"{node}\n")
        (d / "local_cpulist").write_text(NODE_CPUS[node] + "\n")
    for k, cpus in NODE_CPUS.items():
        d = root / "devices" / "system" / "node" / f"node{k}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
    cg = root / "fs" / "cgroup"
    cg.mkdir(parents=True)
    if quota_line is not None:
        (cg / "cpu.max").write_text(quota_line + "\n")
    if v1 is not None:
        (cg / "cpu").mkdir()
        (cg / "cpu" / "cpu.cfs_quota_us").write_text(f"{v1[0]}\n")
        (cg / "cpu" / "cpu.cfs_period_us").write_text(f"{v1[1]}\n")
    return str(root)


@pytest.mark.parametrize("quota", [16, 64, 256])
@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_eight_gpu_node_plan(tmp_path, monkeypatch, quota, n):
    monkeypatch.setenv("S3H_SYSFS_ROOT", fake_node(tmp_path))
    prev = s3.host_numa("local")
    try:
        # the driver's devices 0..N-1; N = 2 and 4 on socket 0, N = 8 on both
        p = s3.host_plan(BDFS[:n], affinity="0-255", cpu_quota=quota)
    finally:
        s3.host_numa(prev)
    cpus = min(256, quota)
    assert p["cpus"] == cpus and p["affinity_cpus"] == 256 and p["devices"] == n
    per = min(16, max(1, cpus // n))
    assert p["staging_threads_per_device"] == per and p["threads"] == per * n
    # the quota is never oversubscribed, on the whole or on a node
    assert not p["oversubscribed"] and p["threads"] <= cpus
    assert not p["node_oversubscribed"]
    for k, d in enumerate(p["per_device"]):
        node = 0 if k < 4 else 1
        assert d["node"] == node and d["bind_node"] == node
        assert d["bind_cpus"] == 128 and d["staging_threads"] == per
        assert (d["bind_first_cpu"], d["bind_last_cpu"]) == ((0, 191) if node == 0 else (64, 255))
    # below the pageable saturation point (6 staging threads per device) only where the quota
    # leaves no more: 16 CPUs over 4 or 8 devices.  Pinned sources need no staging threads.
    assert p["below_saturation"] == (per < 6)
    assert p["below_saturation"] == (quota == 16 and n >= 4)
    # split route: pinned parts give the CPU side every thread; staged sources give each device
    # tg of its share and the CPU side the rest -- never more than the quota, never none
    assert p["split_cpu_threads_pinned"] == cpus
    if p["split_candidates"]:
        assert 1 <= p["split_stage_min"] <= p["split_stage_max"]
        assert p["split_stage_max"] * n < cpus
        assert p["split_cpu_threads_min"] == cpus - p["split_stage_max"] * n >= 1
        assert p["split_cpu_threads_max"] == cpus - p["split_stage_min"] * n
    else:  # 16 CPUs over 8 devices: 2 each, nothing left for a CPU side
        assert quota == 16 and n == 8


def test_plan_reads_the_cgroup_quota(tmp_path, monkeypatch):
    """cpu_quota < 0: the process's cgroup -- cgroup v2 cpu.max or v1 cfs_quota/cfs_period under
    S3H_SYSFS_ROOT/fs/cgroup; "max" or no file means no quota."""
    for quota_line, v1, want in (("1600000 100000", None, 16), ("max 100000", None, 256),
                                 ("650000 100000", None, 7), (None, (6400000, 100000), 64),
                                 (None, (-1, 100000), 256), (None, None, 256)):
        d = tmp_path / f"case{want}_{quota_line is None}_{v1 is None}"
        d.mkdir()
        monkeypatch.setenv("S3H_SYSFS_ROOT", fake_node(d, quota_line, v1))
        p = s3.host_plan(BDFS, affinity="0-255", cpu_quota=-1)
        assert p["cpus"] == want, (quota_line, v1)
        assert p["staging_threads_per_device"] == min(16, max(1, want // 8))


def test_plan_follows_affinity_and_policy(tmp_path, monkeypatch):
    """Only CPUs of the affinity are bound; a device without a NUMA record stays unbound; the
    'off' policy binds nothing; more devices than CPUs are flagged oversubscribed."""
    monkeypatch.setenv("S3H_SYSFS_ROOT", fake_node(tmp_path))
    p = s3.host_plan(BDFS[:2] + [None], affinity="0-7,64-71", cpu_quota=0)
    assert p["cpus"] == 16
    d0, d1, dn = p["per_device"]
    assert d0["bind_cpus"] == 8 and (d0["bind_first_cpu"], d0["bind_last_cpu"]) == (0, 7)
    assert dn["node"] == -1 and dn["bind_cpus"] == 0 and dn["bind_node"] == -1
    prev = s3.host_numa("off")
    try:
        p = s3.host_plan(BDFS, affinity="0-255", cpu_quota=0)
        assert all(d["bind_cpus"] == 0 and d["bind_node"] == -1 for d in p["per_device"])
        assert p["per_device"][5]["node"] == 1  # the record is still read
    finally:
        s3.host_numa(prev)
    p = s3.host_plan(BDFS, affinity="0-3", cpu_quota=0)
    assert p["cpus"] == 4 and p["staging_threads_per_device"] == 1 and p["oversubscribed"]
    with pytest.raises(s3.S3HashError):
        s3.host_plan(BDFS, affinity="x", cpu_quota=0)
    with pytest.raises(s3.S3HashError):
        s3.host_plan([], affinity="0-3", cpu_quota=0)


def test_plan_matches_this_process():
    """With no overrides the plan is the one this process's host calls use (s3h_host_threads)."""
    for n in (1, 2, 3, 8):
        p = s3.host_plan([None] * n)
        per, cpus = s3.host_threads(n)
        assert p["cpus"] == cpus and p["staging_threads_per_device"] == per
        assert p["affinity_cpus"] == len(os.sched_getaffinity(0))


def test_pci_power_cap_from_sysfs(tmp_path, monkeypatch):
    """The POWER kernel policy's input (plan.cpp resolve_kernel): hwmon power1_cap in microwatts
    under the device's PCI function, 0 when the platform has none."""
    root = fake_node(tmp_path)
    hw = tmp_path / "sys" / "bus" / "pci" / "devices" / BDFS[5] / "hwmon" / "hwmon7"
    hw.mkdir(parents=True)
    (hw / "power1_cap").write_text("1400000000\n")
    monkeypatch.setenv("S3H_SYSFS_ROOT", root)
    assert s3.pci_power_cap(BDFS[5]) == 1400.0
    assert s3.pci_power_cap(BDFS[5].upper()) == 1400.0
    assert s3.pci_power_cap(BDFS[0]) == 0.0          # no hwmon directory
    assert s3.pci_power_cap("0000:ff:00.0") == 0.0   # no such function
