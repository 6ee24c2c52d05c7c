"""Random batch shapes through AUTO, every digest vs the oracle.

The plan builder sorts parts by length, groups them, splits the longest into solo workgroups
(capi.hip plan build) and scatters digests back through ``out_idx``; the choice of kernel and
of that layout depends on the part count AND the length distribution.  The fixed-shape tests
cover each kernel's switch points with small uniform parts; here seeded draws mix the part
count (across every AUTO range) with length shapes a real upload produces -- one huge object
among many small ones, two sizes, heavy tails, runs of empty parts -- and compare the whole
batch of SHA-256, MD5 and both-digest results with the oracle (lib/hash sha256.cpp:147-160,
md5.cpp:71-116), bit-exact."""
import numpy as np
import pytest

import s3client_amd as s3

pytestmark = pytest.mark.gpu
MIB = 1 << 20
BUF = 192 * MIB          # device buffer the parts are cut from (parts may overlap)
BUDGET = 160 * MIB       # total bytes per draw, so the oracle stays at ~1 s per draw

COUNT_RANGES = [(1, 64), (65, 2048), (2049, 4096), (4097, 8192), (8193, 28672),
                (28673, 32768), (32769, 65536), (65537, 90000)]
SHAPES = ["one_giant", "bimodal", "lognormal", "empty_runs", "block_edges"]


def _lengths(rng, shape, n):
    if shape == "one_giant":          # one big object, the rest tiny: solo workgroup split
        lens = rng.integers(0, 2000, n)
        lens[rng.integers(0, n)] = rng.integers(8 * MIB, 24 * MIB)
    elif shape == "bimodal":          # full parts plus a short last part per object
        big = int(rng.integers(64 * 1024, 4 * MIB))
        lens = np.where(rng.random(n) < 0.8, big, rng.integers(0, big, n))
    elif shape == "lognormal":        # heavy tail
        lens = np.minimum(rng.lognormal(8, 2.5, n).astype(np.int64), 16 * MIB)
    elif shape == "empty_runs":       # long runs of empty parts between non-empty ones
        lens = rng.integers(0, 300000, n)
        lens[(np.arange(n) // 37) % 3 == 0] = 0
    else:                             # lengths at the 55/56/64-byte padding edges of blocks
        k = rng.integers(0, 2000, n)
        lens = k * 64 + rng.choice([0, 55, 56, 63, 64 - 1, 1], n)
    lens = lens.astype(np.int64)
    total = int(lens.sum())
    if total > BUDGET:                # scale down, keeping the shape (and any empties)
        lens = (lens * (BUDGET / total)).astype(np.int64)
    return np.minimum(lens, BUF)


def _draws(seed, count):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        lo, hi = COUNT_RANGES[i % len(COUNT_RANGES)]
        n = int(rng.integers(lo, hi + 1))
        shape = SHAPES[(i // len(COUNT_RANGES) + i) % len(SHAPES)]
        lens = _lengths(rng, shape, n)
        offs = rng.integers(0, BUF - lens + 1)
        out.append((n, shape, offs.astype(np.uint64), lens.astype(np.uint64)))
    return out


@pytest.fixture(scope="module")
def device_bytes(torch_cuda):
    rng = np.random.default_rng(777)
    host = rng.integers(0, 256, BUF, dtype=np.uint8)
    dev = torch_cuda.from_numpy(host).cuda()
    return host, dev


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_shapes_sha256(torch_cuda, oracle, device_bytes, seed):
    host, dev = device_bytes
    for n, shape, offs, lens in _draws(seed, 16):
        plan = s3.Plan(offs, lens)
        kernel = plan.info()["kernel"]
        plan.close()
        got = s3.sha256_batch_device(dev, offs, lens).cpu().numpy().view(np.uint32)
        want = oracle.batch(host, offs, lens, threads=16)
        bad = np.flatnonzero((got != want).any(axis=1))
        assert bad.size == 0, (n, shape, kernel, bad[:8], lens[bad[:8]])


def test_random_shapes_md5_and_both(torch_cuda, oracle, device_bytes):
    host, dev = device_bytes
    for i, (n, shape, offs, lens) in enumerate(_draws(4, 16)):
        want_m = oracle.md5_batch(host, offs, lens, threads=16)
        if i % 2:
            m5 = s3.md5_batch_device(dev, offs, lens).cpu().numpy().view(np.uint32)
        else:
            sha, m5 = s3.sha256_md5_batch_device(dev, offs, lens)
            m5 = m5.cpu().numpy().view(np.uint32)
            want_s = oracle.batch(host, offs, lens, threads=16)
            bad = np.flatnonzero((sha.cpu().numpy().view(np.uint32) != want_s).any(axis=1))
            assert bad.size == 0, ("sha256", n, shape, bad[:8])
        bad = np.flatnonzero((m5 != want_m).any(axis=1))
        assert bad.size == 0, ("md5", n, shape, bad[:8], lens[bad[:8]])


def test_random_shapes_host_path(torch_cuda, oracle, device_bytes):
    """The same shapes from pageable host memory (H2D slices, staging, tail ramp)."""
    host, _ = device_bytes
    for n, shape, offs, lens in _draws(5, 8):
        views = [host[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]
        got = s3.sha256_batch_host(views)
        want = oracle.batch(host, offs, lens, threads=16)
        bad = np.flatnonzero((got != want).any(axis=1))
        assert bad.size == 0, (n, shape, bad[:8], lens[bad[:8]])
