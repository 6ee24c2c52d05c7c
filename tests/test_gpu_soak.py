"""Randomised soak over every host-facing entry point, every digest vs the oracle.

The fixed-shape tests pin each path's switch points; this one draws batches the way the
shape tests do (part counts across every AUTO kernel range, upload-like length shapes, plus
many small parts and small parts with a few large ones -- the group pipeline and its split
from the slice pipeline) and sends each through the next entry point in turn: device SHA-256 /
MD5 / both, host batches from numpy views, pinned and pageable BufferParts (SHA-256, MD5,
both, verification with corrupted expectations, also on the CPU / split / AUTO routes), file
ranges (SHA-256, both), the routed split and AUTO routes, and streamed objects fed in random
pieces from host memory.  Every
result is checked whole against the oracle (lib/hash sha256.cpp:147-160, md5.cpp:71-116).

S3H_SOAK_SECONDS sets how long it runs (default 20 s: every entry point at least once);
S3H_SOAK_SEED the draw seed.  A failure names the entry point, draw and shape.
"""
import os
import time
from collections import Counter

import numpy as np
import pytest

import s3client_amd as s3
from tests.test_gpu_shapes import BUF, COUNT_RANGES, SHAPES, _lengths

pytestmark = pytest.mark.gpu
MIB = 1 << 20
SOAK_S = float(os.environ.get("S3H_SOAK_SECONDS", "20"))
SEED = int(os.environ.get("S3H_SOAK_SEED", "2024"))
ENTRIES = ["device", "device_md5", "device_dual", "host_views", "host_pinned", "host_pageable",
           "host_dual", "host_md5", "verify", "file", "file_dual", "split", "auto", "stream_host",
           "verify_routed"]
EXTRA_SHAPES = ["many_small", "small_and_large"]


def _draw(rng, i):
    shapes = SHAPES + EXTRA_SHAPES
    shape = shapes[int(rng.integers(0, len(shapes)))]
    if shape == "many_small":       # the group pipeline: thousands of parts <= 64 KiB
        n = int(rng.integers(2049, 20000))
        lens = rng.integers(0, 64 << 10, n)
    elif shape == "small_and_large":  # groups, then the slice pipeline for the large parts
        n = int(rng.integers(2049, 6000))
        lens = rng.integers(0, 32 << 10, n)
        lens[rng.integers(0, n, 3)] = rng.integers(2 * MIB, 12 * MIB, 3)
    else:
        lo, hi = COUNT_RANGES[i % len(COUNT_RANGES)]
        n = int(rng.integers(lo, hi + 1))
        lens = _lengths(rng, shape, n)
    lens = lens.astype(np.int64)
    if lens.sum() > 256 * MIB:      # keep the oracle at well under a second per draw
        lens = (lens * (256 * MIB / lens.sum())).astype(np.int64)
    lens = np.minimum(lens, BUF)
    offs = rng.integers(0, BUF - lens + 1)
    return n, shape, offs.astype(np.uint64), lens.astype(np.uint64)


@pytest.fixture(scope="module")
def soak_data(torch_cuda, tmp_path_factory):
    torch = torch_cuda
    rng = np.random.default_rng(4711)
    host = rng.integers(0, 256, BUF, dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    pinned = torch.empty(BUF, dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = host
    path = tmp_path_factory.mktemp("soak") / "src.bin"
    host.tofile(path)
    return host, dev, pinned, str(path)


def _stream_pieces(rng, offs, lens):
    """Each message cut at random points into R pieces (some empty): per update, the pieces'
    offsets and lengths."""
    r = int(rng.integers(1, 6))
    cuts = np.sort(rng.random((len(lens), r - 1)) * lens[:, None].astype(np.float64), axis=1).astype(np.uint64)
    cuts = np.concatenate([np.zeros((len(lens), 1), np.uint64), cuts, lens[:, None]], axis=1)
    return [(offs + cuts[:, k], cuts[:, k + 1] - cuts[:, k]) for k in range(r)]


def _run(entry, rng, torch, oracle, data, offs, lens, want_sha):
    """Runs one entry point on the draw; returns a list of (what, got, want) to compare."""
    host, dev, pinned, path = data
    src = pinned if rng.random() < 0.5 else host
    out = []
    if entry == "device":
        got = s3.sha256_batch_device(dev, offs, lens).cpu().numpy().view(np.uint32)
        out.append(("sha256", got, want_sha()))
    elif entry == "device_md5":
        got = s3.md5_batch_device(dev, offs, lens).cpu().numpy().view(np.uint32)
        out.append(("md5", got, oracle.md5_batch(host, offs, lens, threads=16)))
    elif entry == "device_dual":
        sha, m5 = s3.sha256_md5_batch_device(dev, offs, lens)
        torch.cuda.synchronize()
        out.append(("sha256", sha.cpu().numpy().view(np.uint32), want_sha()))
        out.append(("md5", m5.cpu().numpy().view(np.uint32), oracle.md5_batch(host, offs, lens, threads=16)))
    elif entry == "host_views":
        views = [host[int(o):int(o) + int(n)] for o, n in zip(offs, lens)]
        out.append(("sha256", s3.sha256_batch_host(views), want_sha()))
    elif entry in ("host_pinned", "host_pageable"):
        buf = pinned if entry == "host_pinned" else host
        out.append(("sha256", s3.sha256_batch_host(s3.BufferParts(buf, offs, lens)), want_sha()))
    elif entry == "host_dual":
        sha, m5 = s3.sha256_md5_batch_host(s3.BufferParts(src, offs, lens))
        out.append(("sha256", sha, want_sha()))
        out.append(("md5", m5, oracle.md5_batch(host, offs, lens, threads=16)))
    elif entry == "host_md5":
        got = s3.md5_batch_host(s3.BufferParts(src, offs, lens))
        out.append(("md5", got, oracle.md5_batch(host, offs, lens, threads=16)))
    elif entry == "verify":
        exp = want_sha().copy()
        bad = rng.random(len(lens)) < 0.01
        exp[bad, int(rng.integers(0, 8))] ^= np.uint32(1 << int(rng.integers(0, 32)))
        mism = s3.verify_batch_host(s3.BufferParts(src, offs, lens), exp)
        out.append(("mismatch mask", mism[:, None], bad[:, None]))
    elif entry == "file":
        out.append(("sha256", s3.sha256_file_parts(path, offs, lens), want_sha()))
    elif entry == "file_dual":
        sha, m5 = s3.sha256_md5_file_parts(path, offs, lens)
        out.append(("sha256", sha, want_sha()))
        out.append(("md5", m5, oracle.md5_batch(host, offs, lens, threads=16)))
    elif entry in ("split", "auto"):
        got, taken = s3.sha256_batch_routed(s3.BufferParts(src, offs, lens), route=entry)
        assert taken in ("gpu", "cpu", "split"), taken
        assert entry == "auto" or taken == ("split" if len(lens) > 1 else "gpu"), taken
        out.append((f"sha256 ({taken})", got, want_sha()))
    elif entry == "verify_routed":
        exp = want_sha().copy()
        bad = rng.random(len(lens)) < 0.01
        exp[bad, int(rng.integers(0, 8))] ^= np.uint32(1 << int(rng.integers(0, 32)))
        route = ("cpu", "split", "auto")[int(rng.integers(0, 3))]
        mism, taken = s3.verify_batch_routed(s3.BufferParts(src, offs, lens), exp, route=route)
        out.append((f"mismatch mask ({route} -> {taken})", mism[:, None], bad[:, None]))
    elif entry == "stream_host":
        with s3.Stream(len(lens)) as st:
            for po, pl in _stream_pieces(rng, offs, lens):
                st.update(s3.BufferParts(src, po, pl))
            got = st.final()
        out.append(("sha256", got, want_sha()))
    else:
        raise AssertionError(entry)
    return out


def test_soak_every_entry_point(torch_cuda, oracle, soak_data):
    torch = torch_cuda
    host = soak_data[0]
    rng = np.random.default_rng(SEED)
    counts, parts = Counter(), Counter()
    t_end = time.monotonic() + SOAK_S
    t_note = time.monotonic() + 30
    i = 0
    while i < len(ENTRIES) or time.monotonic() < t_end:
        if time.monotonic() > t_note:  # a progress line every 30 s (seen with -s)
            print(f"soak: {i} draws, {sum(parts.values())} parts so far", flush=True)
            t_note += 30
        entry = ENTRIES[i % len(ENTRIES)]
        n, shape, offs, lens = _draw(rng, i)
        memo = {}

        def want_sha():
            if "sha" not in memo:
                memo["sha"] = oracle.batch(host, offs, lens, threads=16)
            return memo["sha"]

        for what, got, want in _run(entry, rng, torch, oracle, soak_data, offs, lens, want_sha):
            bad = np.flatnonzero((np.asarray(got) != np.asarray(want)).any(axis=1))
            assert bad.size == 0, (entry, what, "draw", i, "seed", SEED, shape, n, bad[:8], lens[bad[:8]])
        counts[entry] += 1
        parts[entry] += n
        i += 1
    print(f"soak: {i} draws in {SOAK_S:.0f} s, seed {SEED}: " +
          ", ".join(f"{e} {counts[e]} ({parts[e]} parts)" for e in ENTRIES))
