"""NUMA placement of the host path on the GPU box: the device's node
from sysfs, pinned staging and copy threads placed there (or where the policy says), pinned
buffers on a chosen node, and bit-exact digests whatever the placement."""
import os
import subprocess
import sys

import numpy as np
import pytest

import s3client_amd as s3

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIB = 1 << 20


def _allowed_nodes():
    with open("/proc/self/status") as f:
        s = next(l.split(":", 1)[1].strip() for l in f if l.startswith("Mems_allowed_list"))
    out = []
    for part in s.split(","):
        lo, _, hi = part.partition("-")
        out += list(range(int(lo), int(hi or lo) + 1))
    return out


def _parts(rng, n=48, L=2 * MIB + 77):
    data = rng.integers(0, 256, n * L, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    lens = np.full(n, L, dtype=np.uint64)
    return data, offs, lens


def test_device_node_matches_sysfs(torch_cuda):
    bdf = s3.device_pci_bus_id(0)
    with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
        want = max(-1, int(f.read()))
    got = s3.device_numa(0)
    assert got["node"] == want
    assert got == {k: v for k, v in s3.pci_numa(bdf).items() if k != "usable_cpus"}


def test_staging_and_threads_follow_the_policy(torch_cuda, oracle):
    """Pageable parts stage through the pinned ring: its pages and the copy threads land on
    the device's node by default, on a forced node when asked, unbound with "off"; the digests
    never change."""
    rng = np.random.default_rng(51)
    data, offs, lens = _parts(rng)
    want = oracle.batch(data, offs, lens)
    views = [data[int(o):int(o) + int(n)] for o, n in zip(offs, lens)]  # pageable
    dn = s3.device_numa(0)["node"]
    prev = s3.host_numa("local")
    try:
        s3.trim()
        assert np.array_equal(s3.sha256_batch_host(views, ndevices=1), want)
        info = s3.host_numa_info(0)
        assert info["device_node"] == dn and info["target_node"] == dn
        if dn >= 0:
            assert info["staging_node"] == dn, info
            assert info["bound_cpus"] > 0 and info["threads_node"] == dn, info
        for node in _allowed_nodes():
            s3.host_numa(node)
            assert np.array_equal(s3.sha256_batch_host(views, ndevices=1), want)
            info = s3.host_numa_info(0)
            assert info["target_node"] == node and info["staging_node"] == node, info
        s3.host_numa("off")
        assert np.array_equal(s3.sha256_batch_host(views, ndevices=1), want)
        info = s3.host_numa_info(0)
        assert info["target_node"] == -1 and info["threads_node"] == -1 and info["bound_cpus"] == 0
    finally:
        s3.host_numa(prev)
        s3.trim()


@pytest.mark.parametrize("where", ["local", "remote", "runtime"])
def test_pinned_buffer_on_a_node_hashes_as_pinned(torch_cuda, oracle, where):
    """s3h_host_alloc pages sit on the node asked for; the host path treats them as pinned
    (direct 2-D DMA, no staging) and the digests equal the oracle's."""
    dn = s3.device_numa(0)["node"]
    others = [k for k in _allowed_nodes() if k != dn]
    node = {"local": dn, "remote": others[0] if others else dn, "runtime": -1}[where]
    rng = np.random.default_rng(52)
    data, offs, lens = _parts(rng, n=40, L=MIB)
    buf = s3.PinnedBuffer(data.size, node)
    buf.array[:] = data
    if node >= 0:
        assert s3.mem_node(buf.array) == node
        assert s3.mem_node(buf.array[-1:]) == node
    got = s3.sha256_batch_host(s3.BufferParts(buf.array, offs, lens), ndevices=1)
    assert np.array_equal(got, oracle.batch(data, offs, lens))
    buf.close()


def test_registered_buffer_takes_the_pinned_path(torch_cuda):
    """The trace line (S3H_TRACE_HOST) of a call on s3h_host_alloc memory says "pinned 2-D":
    hipHostRegister'd pages are DMA'd directly, never re-staged."""
    code = ("import numpy as np, s3client_amd as s3\n"
            "n, L = 16, 1 << 20\n"
            "b = s3.PinnedBuffer(n * L, s3.device_numa(0)['node'])\n"
            "b.array[:] = 7\n"
            "offs = np.arange(n, dtype=np.uint64) * np.uint64(L)\n"
            "s3.sha256_batch_host(s3.BufferParts(b.array, offs, np.full(n, L, np.uint64)), 1)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       env={**os.environ, "S3H_TRACE_HOST": "1"}, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "pinned 2-D" in r.stderr, r.stderr


def test_strict_and_preferred_placement(torch_cuda, oracle):
    """Advisor r5: staging and s3h_host_alloc PREFER their node (a short node spills to another
    instead of OOM-killing the process); S3H_HOST_ALLOC_STRICT binds, after checking the node's
    free memory -- a request beyond it fails cleanly with S3H_ENOMEM, before any page is touched."""
    dn = s3.device_numa(0)["node"]
    node = dn if dn >= 0 else 0
    rng = np.random.default_rng(53)
    data, offs, lens = _parts(rng, n=16, L=MIB)
    for strict in (False, True):
        buf = s3.PinnedBuffer(data.size, node, strict=strict)
        buf.array[:] = data
        assert s3.mem_node(buf.array) == node and s3.mem_node(buf.array[-1:]) == node
        got = s3.sha256_batch_host(s3.BufferParts(buf.array, offs, lens), ndevices=1)
        assert np.array_equal(got, oracle.batch(data, offs, lens))
        buf.close()
    with pytest.raises(s3.S3HashError) as e:  # 64 TiB on one node: refused, not OOM-killed
        s3.PinnedBuffer(64 << 40, node, strict=True)
    assert e.value.code == -4 and "strict" in str(e.value)
    with pytest.raises(s3.S3HashError):
        s3._native.check(s3._native.lib().s3h_host_alloc_ex(node, 4096, 8, None))
