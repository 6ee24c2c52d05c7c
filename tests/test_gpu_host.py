"""Host-resident path (H2D included) under the conditions a real uploader creates: cached
per-device contexts that grow and are trimmed, many pageable parts, concurrent callers, parts
read from a file, and plans launched on two streams at once.  Every digest vs the oracle or
the lib/hash goldens (bit-exact)."""
import os
import threading
import time

import numpy as np
import pytest

import s3client_amd as s3

pytestmark = pytest.mark.gpu
MIB = 1 << 20


def _free(torch):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return torch.cuda.mem_get_info()[0]


def test_context_grows_keeps_small_ring_and_trims(torch_cuda, oracle):
    """Small call, then a larger one (the cached ring and plans grow), then one whose HBM ring
    exceeds the 1 GiB keep limit (freed when the call returns), then s3h_trim (all freed)."""
    torch = torch_cuda
    # The process's first host-path call also loads the code object and the runtime's own
    # device allocations (~170 MiB, which no trim returns): take the baseline after one.
    s3.sha256_batch_host([np.zeros(1, dtype=np.uint8)])
    s3.trim()
    free0 = _free(torch)
    rng = np.random.default_rng(51)
    small = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 5000, 64)]
    assert np.array_equal(s3.sha256_batch_host(small),
                          np.stack([oracle.sha256(p.tobytes()) for p in small]))
    larger = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 300000, 1500)]
    assert np.array_equal(s3.sha256_batch_host(larger),
                          np.stack([oracle.sha256(p.tobytes()) for p in larger]))
    kept = free0 - _free(torch)
    # small ring + plans stay cached (a few MiB below zero: allocations of earlier tests in this
    # process that the runtime released meanwhile)
    assert -64 * MIB <= kept < 256 * MIB, kept
    # pinned, non-uniform parts -> 2 MiB slices: ring = 3 x 200 x 2 MiB = 1.2 GiB > 1 GiB
    pinned = torch.empty(200 * (2 * MIB + 64), dtype=torch.uint8, pin_memory=True)
    h = pinned.numpy()
    h[:] = rng.integers(0, 256, h.size, dtype=np.uint8)
    views = [h[i * (2 * MIB + 64): i * (2 * MIB + 64) + 2 * MIB + (i % 7)] for i in range(200)]
    want = oracle.batch(h, [i * (2 * MIB + 64) for i in range(200)], [v.size for v in views])
    assert np.array_equal(s3.sha256_batch_host(views), want)
    after_big = free0 - _free(torch)
    assert after_big < 512 * MIB, after_big       # the 1.2 GiB ring was not kept
    s3.trim()
    trimmed = free0 - _free(torch)
    assert trimmed < 64 * MIB, trimmed


def test_pageable_parts_beyond_staging_slot_cap(torch_cuda, oracle):
    """> 8,192 pageable parts: slices shrink below 4 KiB so the pinned staging slot stays at
    32 MiB; > 524,288 parts: per-part pageable DMAs.  Both vs the oracle."""
    rng = np.random.default_rng(52)
    n = 10000
    lens = rng.integers(0, 9000, n)
    lens[:3] = [0, 55, 4097]
    buf = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    views = [buf[o:o + L] for o, L in zip(offs, lens)]
    assert np.array_equal(s3.sha256_batch_host(views), oracle.batch(buf, offs, lens))
    n = 530000
    lens = rng.integers(0, 40, n)
    buf = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    views = [buf[o:o + L] for o, L in zip(offs, lens)]
    got = s3.sha256_batch_host(views)
    idx = rng.choice(n, 3000, replace=False)
    assert np.array_equal(got[idx], oracle.batch(buf, offs[idx], lens[idx]))


def test_concurrent_host_callers(torch_cuda, oracle, golden):
    """Four threads hash at the same time (ctypes drops the GIL), as upload.cpp:136-140 runs one
    std::async job per part group: their calls are merged into shared batches.  Each thread's
    digests vs the transfer-test goldens / the oracle."""
    t = golden["transfer"]
    data = (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8)
    views = [data[p["offset"]:p["offset"] + p["size"]] for p in t["parts"]]
    want_x = [p["digest"] for p in t["parts"]]
    rng = np.random.default_rng(53)
    sets = [[rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 200000, 300)]
            for _ in range(3)]
    want_r = [np.stack([oracle.sha256(p.tobytes()) for p in s]) for s in sets]
    errors, results = [], {}

    def job(k):
        try:
            for _ in range(3):
                if k == 0:
                    results[k] = s3.digests_to_text(s3.sha256_batch_host(views))
                else:
                    results[k] = s3.sha256_batch_host(sets[k - 1])
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=job, args=(k,)) for k in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    assert results[0] == want_x
    for k in range(1, 4):
        assert np.array_equal(results[k], want_r[k - 1]), k


def test_sixteen_concurrent_callers_merged(torch_cuda, oracle):
    """16 job threads (the upload.cpp:136-140 shape at -j 16), three rounds each on their own
    ragged parts: the calls meet in the device's queue and run as merged batches, each caller
    getting exactly its own digests back (vs the oracle every round); s3h_trim then frees the
    device's context."""
    torch = torch_cuda
    s3.trim()
    free0 = _free(torch)
    rng = np.random.default_rng(57)
    sets = [[rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 120000, 40)]
            for _ in range(16)]
    want = [np.stack([oracle.sha256(p.tobytes()) for p in ps]) for ps in sets]
    errors, bad = [], []

    def job(k):
        try:
            for r in range(3):
                if not np.array_equal(s3.sha256_batch_host(sets[k]), want[k]):
                    bad.append((k, r))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=job, args=(k,)) for k in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors and not bad, (errors, bad)
    s3.trim()
    assert free0 - _free(torch) < 64 * MIB


def test_concurrent_mixed_sources_and_algorithms(torch_cuda, oracle, tmp_path):
    """Concurrent calls of different kinds on one device: file ranges and memory parts
    (SHA-256, merged into one batch of per-part references) beside SHA-256 + MD5 calls (a
    different algorithm set: their own batches).  Every digest vs the oracle / hashlib."""
    import hashlib
    rng = np.random.default_rng(58)
    data = np.frombuffer(rng.bytes(8 * MIB), dtype=np.uint8)
    path = tmp_path / "mixed.bin"
    data.tofile(path)
    fo = rng.integers(0, 7 * MIB, 50)
    fl = rng.integers(0, MIB, 50)
    mem = [[rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 200000, 30)]
           for _ in range(3)]
    want_f = oracle.batch(data, fo, fl)
    want_m = [np.stack([oracle.sha256(p.tobytes()) for p in ps]) for ps in mem]
    want_md5 = [[hashlib.md5(p.tobytes()).hexdigest() for p in ps] for ps in mem]
    errors, bad = [], []

    def job(k):
        try:
            for r in range(2):
                if k == 0:
                    ok = np.array_equal(s3.sha256_file_parts(str(path), fo, fl), want_f)
                elif k <= 3:
                    ok = np.array_equal(s3.sha256_batch_host(mem[k - 1]), want_m[k - 1])
                else:
                    sha, md5 = s3.sha256_md5_batch_host(mem[k - 4])
                    ok = (np.array_equal(sha, want_m[k - 4])
                          and s3.digests_to_text(md5, 4) == want_md5[k - 4])
                if not ok:
                    bad.append((k, r))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=job, args=(k,)) for k in range(7)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors and not bad, (errors, bad)


def test_concurrent_bad_call_fails_alone(torch_cuda, oracle, tmp_path):
    """A file-range call with a part past the end of the file fails by itself (checked before
    it can join a merged batch) while concurrent good calls on the device succeed."""
    rng = np.random.default_rng(59)
    data = np.frombuffer(rng.bytes(2 * MIB), dtype=np.uint8)
    path = tmp_path / "bad.bin"
    data.tofile(path)
    parts = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 300000, 40)]
    want = np.stack([oracle.sha256(p.tobytes()) for p in parts])
    res = {}

    def good(k):
        res[k] = all(np.array_equal(s3.sha256_batch_host(parts), want) for _ in range(3))

    def bad():
        try:
            s3.sha256_file_parts(str(path), [0, 2 * MIB - 5], [100, 10])
            res["bad"] = "no error"
        except s3.S3HashError as e:
            res["bad"] = str(e)

    th = [threading.Thread(target=good, args=(k,)) for k in range(4)] + [threading.Thread(target=bad)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert all(res[k] for k in range(4)), res
    assert "past the end" in res["bad"], res


def test_merged_batch_failure_is_rerun_per_caller(torch_cuda, oracle, tmp_path):
    """A file shrinks AFTER its call passed the open-time range check and queued behind a busy
    device: the merged batch it joins fails on the short read.  That batch is re-run one
    request at a time (capi.hip run_batch), so the concurrent memory call queued with it gets
    its digests and OK, and only the file call fails, with its own message."""
    rng = np.random.default_rng(61)
    path = tmp_path / "shrinks.bin"
    np.frombuffer(rng.bytes(4 * MIB), dtype=np.uint8).tofile(path)
    busy = [np.frombuffer(rng.bytes(8 * MIB), dtype=np.uint8) for _ in range(96)]
    mem = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(1, 200000, 24)]
    want = np.stack([oracle.sha256(p.tobytes()) for p in mem])
    res = {}

    def run(name, fn):
        try:
            res[name] = fn()
        except s3.S3HashError as e:
            res[name] = e

    t_busy = threading.Thread(target=run, args=("busy", lambda: s3.sha256_batch_host(busy)))
    t_file = threading.Thread(target=run, args=("file", lambda: s3.sha256_file_parts(
        str(path), [0, 2 * MIB], [1 * MIB, 2 * MIB])))
    t_mem = threading.Thread(target=run, args=("mem", lambda: s3.sha256_batch_host(mem)))
    t_busy.start()
    time.sleep(0.03)   # the busy call leads the device queue
    t_file.start()
    time.sleep(0.03)   # the file call passed its range check and waits in the queue
    os.truncate(path, 3 * MIB)
    t_mem.start()
    for t in (t_busy, t_file, t_mem):
        t.join()
    assert not isinstance(res["busy"], Exception), res["busy"]
    assert not isinstance(res["mem"], Exception), res["mem"]
    assert np.array_equal(res["mem"], want)
    # the busy call holds the device for >= one 8 MiB chain (~120 ms), so the file call ran
    # after the truncation -- merged with the memory call, then alone -- and failed by itself
    assert isinstance(res["file"], s3.S3HashError), res["file"]
    assert "reading a part failed" in str(res["file"]), res["file"]


def test_file_parts_beyond_staging_cap(torch_cuda, oracle, tmp_path):
    """More file ranges than 64-B slices of the 128 MiB staging slot hold (2,097,152): the
    shard runs in passes of that many parts, so the pinned staging ring stays at 384 MiB
    (capi.hip run_host_shard_passes).  3,000 sampled digests vs the oracle."""
    rng = np.random.default_rng(62)
    data = np.frombuffer(rng.bytes(8 * MIB), dtype=np.uint8)
    path = tmp_path / "many.bin"
    data.tofile(path)
    n = 2_100_000
    offs = rng.integers(0, 8 * MIB - 64, n).astype(np.uint64)
    lens = rng.integers(0, 64, n).astype(np.uint64)
    got = s3.sha256_file_parts(str(path), offs, lens)
    idx = np.concatenate([rng.choice(n, 2990, replace=False), np.arange(n - 10, n)])
    assert np.array_equal(got[idx], oracle.batch(data, offs[idx], lens[idx]))


def test_file_parts_transfer_geometry(torch_cuda, golden, tmp_path):
    """s3h_sha256_file_parts: the transfer test's file, parts as (offset, size) ranges sliced by
    lib/src/upload.cpp geometry (3 jobs x 2 parts), preads straight into pinned staging."""
    t = golden["transfer"]
    path = tmp_path / "xfer.bin"
    (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8).tofile(path)
    offs = [p["offset"] for p in t["parts"]]
    sizes = [p["size"] for p in t["parts"]]
    for sl in (0, 64 << 10):
        got = s3.digests_to_text(s3.sha256_file_parts(str(path), offs, sizes, slice_bytes=sl))
        assert got == [p["digest"] for p in t["parts"]], sl
    with pytest.raises(s3.S3HashError):  # a part past the end of the file
        s3.sha256_file_parts(str(path), [t["size"] - 10], [100])
    with pytest.raises(s3.S3HashError):
        s3.sha256_file_parts(str(tmp_path / "missing.bin"), [0], [1])


def test_file_parts_many_parts(torch_cuda, oracle, tmp_path):
    """s3h_sha256_file_parts over 3,000 ragged ranges (incl. empty, overlapping and file-final
    parts; 128 MiB file staging slots) vs the oracle; a range past the end of the file is
    S3H_EINVAL."""
    rng = np.random.default_rng(56)
    size = 40 * MIB + 13
    data = np.frombuffer(rng.bytes(size), dtype=np.uint8)
    path = tmp_path / "many.bin"
    data.tofile(path)
    n = 3000
    lens = rng.integers(0, 30000, n)
    offs = rng.integers(0, size - 30000, n)
    lens[:3] = [0, 1, 64]
    offs[n - 1], lens[n - 1] = size - 777, 777
    got = s3.sha256_file_parts(str(path), offs, lens)
    assert np.array_equal(got, oracle.batch(data, offs, lens, threads=16))
    bad_offs = offs.copy()
    bad_offs[5] = size - 10
    bad_lens = lens.copy()
    bad_lens[5] = 100
    with pytest.raises(s3.S3HashError):
        s3.sha256_file_parts(str(path), bad_offs, bad_lens)


def test_dual_digest_file_parts(torch_cuda, golden, tmp_path):
    """s3h_sha256_md5_file_parts: the transfer test's file as its six (offset, size) parts --
    SHA-256 vs the lib/hash goldens, MD5s vs md5_file's and the multipart ETag -- and 2,500
    ragged ranges of a random file vs hashlib (both digests, each slice read once)."""
    import hashlib
    t = golden["transfer"]
    path = tmp_path / "xfer.bin"
    (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8).tofile(path)
    sha, m5 = s3.sha256_md5_file_parts(str(path), [p["offset"] for p in t["parts"]],
                                       [p["size"] for p in t["parts"]])
    assert s3.digests_to_text(sha) == [p["digest"] for p in t["parts"]]
    assert s3.digests_to_text(m5, 4) == [p["digest"] for p in golden["md5"]["transfer"]]
    assert s3.multipart_etag(m5) == golden["md5"]["transfer_etag"]
    rng = np.random.default_rng(60)
    size = 24 * MIB + 5
    data = np.frombuffer(rng.bytes(size), dtype=np.uint8)
    path2 = tmp_path / "dual.bin"
    data.tofile(path2)
    n = 2500
    lens = rng.integers(0, 20000, n)
    offs = rng.integers(0, size - 20000, n)
    lens[:4] = [0, 55, 56, 64]
    sha, m5 = s3.sha256_md5_file_parts(str(path2), offs, lens)
    views = [data[o:o + L].tobytes() for o, L in zip(offs, lens)]
    assert s3.digests_to_text(sha) == [hashlib.sha256(v).hexdigest() for v in views]
    assert s3.digests_to_text(m5, 4) == [hashlib.md5(v).hexdigest() for v in views]


def test_two_plans_on_two_streams(torch_cuda, oracle):
    """Two device-resident plans launched concurrently on two torch streams."""
    torch = torch_cuda
    rng = np.random.default_rng(54)
    bufs, plans, outs, wants = [], [], [], []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for k, n in enumerate((1000, 6000)):
        lens = rng.integers(0, 70000, n)
        offs = np.concatenate([[0], np.cumsum(lens + 5)[:-1]])
        host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
        bufs.append(torch.from_numpy(host).cuda())
        plans.append(s3.Plan(offs, lens))
        outs.append(torch.zeros((n, 8), dtype=torch.int32, device="cuda"))
        wants.append(oracle.batch(host, offs, lens))
    torch.cuda.synchronize()
    for k in range(2):
        plans[k].launch(bufs[k], outs[k], streams[k])
    torch.cuda.synchronize()
    for k in range(2):
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32), wants[k]), k
        plans[k].close()


def test_sharded_host_batch_on_repeated_device(torch_cuda, oracle):
    """The multi-device host path (one host thread per shard, part i on shard i % N, digests
    reassembled in part order) exercised on one GPU by listing it 3 times: the three shards
    meet in the device's queue and run as one merged batch."""
    rng = np.random.default_rng(55)
    parts = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 300000, 301)]
    want = np.stack([oracle.sha256(p.tobytes()) for p in parts])
    assert np.array_equal(s3.sha256_batch_host_on(parts, [0, 0, 0]), want)
    assert np.array_equal(s3.sha256_batch_host_on(parts[:2], [0, 0, 0, 0]), want[:2])
    with pytest.raises(s3.S3HashError):
        s3.sha256_batch_host_on(parts, [0, 99])


def test_host_batch_shared_simd_kernel_range(torch_cuda, oracle):
    """4,097-8,192 parts (AUTO = the shared-SIMD skew kernel, one 32-part workgroup per CU)
    from pinned memory at a constant stride (2-D copies, 256 KiB slices) and from pageable
    parts (staged slices): every slice is a resumable launch of that kernel (the "throughput"
    policy: the default "power" policy may pick skewp on a power-capped board)."""
    torch = torch_cuda
    prev = s3.kernel_policy("throughput")
    try:
        _host_shared_simd_range(torch, oracle)
    finally:
        s3.kernel_policy(prev)


def _host_shared_simd_range(torch, oracle):
    assert s3.Plan([0] * 4500, [1] * 4500).info()["kernel"] == "skews"
    rng = np.random.default_rng(53)
    n, stride = 4500, 600_000  # 3 slices per part
    pinned = torch.empty(n * stride, dtype=torch.uint8, pin_memory=True)
    h = pinned.numpy()
    h[:] = np.frombuffer(rng.bytes(h.size), dtype=np.uint8)
    views = [h[i * stride: i * stride + stride] for i in range(n)]
    want = oracle.batch(h, [i * stride for i in range(n)], [stride] * n, threads=16)
    assert np.array_equal(s3.sha256_batch_host(views), want)
    lens = rng.integers(0, 70000, 5000)
    buf = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    views = [buf[o:o + L] for o, L in zip(offs, lens)]
    assert np.array_equal(s3.sha256_batch_host(views), oracle.batch(buf, offs, lens, threads=16))


def test_device_queue_soak_mixed_calls(torch_cuda, tmp_path):
    """Eight threads, 12 random host calls each -- SHA-256 from memory or file ranges,
    SHA-256 + MD5, download verification with a planted mismatch -- all meeting in the
    device's queue in random combinations; every result vs hashlib."""
    import hashlib
    rng0 = np.random.default_rng(63)
    data = np.frombuffer(rng0.bytes(6 * MIB), dtype=np.uint8)
    path = tmp_path / "soak.bin"
    data.tofile(path)
    errors = []

    def job(k):
        rng = np.random.default_rng(100 + k)
        try:
            for r in range(12):
                n = int(rng.integers(1, 400))
                lens = rng.integers(0, 40000, n)
                offs = rng.integers(0, data.size - 40000, n)
                views = [data[o:o + L] for o, L in zip(offs, lens)]
                sha = [hashlib.sha256(v.tobytes()).hexdigest() for v in views]
                kind = int(rng.integers(0, 4))
                if kind == 0:
                    ok = s3.digests_to_text(s3.sha256_batch_host(views)) == sha
                elif kind == 1:
                    ok = s3.digests_to_text(s3.sha256_file_parts(str(path), offs, lens)) == sha
                elif kind == 2:
                    a, b = s3.sha256_md5_batch_host(views)
                    ok = (s3.digests_to_text(a) == sha and s3.digests_to_text(b, 4) ==
                          [hashlib.md5(v.tobytes()).hexdigest() for v in views])
                else:
                    want = np.stack([np.frombuffer(bytes.fromhex(h), dtype=np.uint32) for h in sha])
                    bad = int(rng.integers(0, n))
                    want[bad, 0] ^= 1
                    mism = s3.verify_batch_host(views, want)
                    ok = list(np.flatnonzero(mism)) == [bad]
                if not ok:
                    errors.append(f"thread {k} call {r} kind {kind} n {n}")
        except Exception as e:  # pragma: no cover - reported below
            errors.append(f"thread {k}: {e!r}")

    th = [threading.Thread(target=job, args=(k,)) for k in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors


def test_route_auto_by_batch_shape(torch_cuda, oracle, golden, tmp_path):
    """S3H_ROUTE_AUTO on a real GPU: the measured model is sane; 1,024 x 8 MiB C2 parts (pinned,
    the bench metric's shape) go to the GPU -- with the CPU drop-in beside it (the split
    route) when the model says so -- and 8 x 8 MiB parts (a per-job batch of
    upload.cpp:89-110) go wherever the model estimates -- on a host with a few SHA-NI cores,
    the CPU.  Every digest equals the GPU-forced path's and the lib/hash fixtures."""
    torch = torch_cuda
    m = s3.route_model()
    assert 20e6 < m["chain_bytes_per_s"] < 200e6, m   # one skew chain: ~69 MB/s at 2.4 GHz
    assert m["h2d_bytes_per_s"] > 5e9 and m["cpu_bytes_per_s"] > 50e6, m
    assert 0 < m["call_s"] < 0.05 and m["cpu_threads"] >= 1 and m["devices"] >= 1, m
    n, L = 1024, 8 * MIB
    lens = np.full(n, L, dtype=np.uint64)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    dev = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    s3.generate_parts(dev, offs, lens, np.arange(n), 20241008)
    host = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    host.copy_(dev)
    del dev
    _free(torch)
    h = host.numpy()
    views = [h[i * L:(i + 1) * L] for i in range(n)]
    fx = {e["p"]: e["digest"] for e in golden["c2_parts"]}
    want_route, g, c = s3.route_estimate([L] * n, m)
    assert want_route == "gpu", (g, c, m)
    k, _, split_s = s3.route_split_estimate([L] * n, m)
    got, taken = s3.sha256_batch_routed(views, route="auto")
    # pinned C2 parts: the split (the CPU drop-in on part of them at once) when it is estimated
    # 5 % faster than the GPU alone -- on the box's 16 SHA-NI threads it is
    assert taken == ("split" if split_s < 0.95 * min(g, c) else "gpu"), (g, c, k, split_s)
    assert all(s3.hash_to_text(got[p]) == d for p, d in fx.items())
    small = views[:8]
    want_route, g, c = s3.route_estimate([L] * 8, m)
    got8, taken = s3.sha256_batch_routed(small, route="auto")
    assert taken == want_route, (g, c)
    assert np.array_equal(got8, got[:8])
    gpu8, taken = s3.sha256_batch_routed(small, route="gpu")
    assert taken == "gpu" and np.array_equal(gpu8, got[:8])
    # file ranges: the same eight parts from a file, both routes
    path = tmp_path / "parts.bin"
    h[:8 * L].tofile(path)
    for route in ("auto", "cpu", "gpu"):
        f8, taken = s3.sha256_file_parts_routed(str(path), offs[:8], lens[:8], route=route)
        assert np.array_equal(f8, got[:8]), route
    del host, h, views


def test_route_auto_near_the_faster_route(torch_cuda):
    """AUTO is within 10 % of the faster forced route at n = 128 (CPU side of the crossover
    on the box's 16 SHA-NI threads) and n = 1,024 (GPU side), pinned 8 MiB parts: median of
    three alternating calls per route (tools/route_sweep.py covers n = 8 ... 1,024, pinned and
    pageable: profiles/r05_route_sweep.json).  The model's CPU rate is the measured
    all-threads rate, not threads x one thread."""
    import time
    torch = torch_cuda
    m = s3.route_model()
    assert 0 < m["cpu_all_bytes_per_s"] <= m["cpu_threads"] * m["cpu_bytes_per_s"] * 1.05, m
    assert m["staged_bytes_per_s"] > 1e9, m
    n, L = 1024, 8 * MIB
    lens = np.full(n, L, dtype=np.uint64)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    dev = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    s3.generate_parts(dev, offs, lens, np.arange(n), 20241008)
    ref = s3.sha256_batch_device(dev, offs, lens).cpu().numpy().view(np.uint32)
    buf = s3.PinnedBuffer(n * L, s3.device_numa(0)["node"])
    torch.from_numpy(buf.array).copy_(dev)
    del dev
    _free(torch)
    for k in (128, 1024):
        parts = s3.BufferParts(buf.array, offs[:k], lens[:k])
        t = {r: [] for r in ("gpu", "cpu", "auto")}
        for rep in range(4):
            for r in t:
                t0 = time.perf_counter()
                d, taken = s3.sha256_batch_routed(parts, ndevices=1, route=r)
                if rep:
                    t[r].append(time.perf_counter() - t0)
                assert np.array_equal(d, ref[:k]), (k, r)
        med = {r: float(np.median(v)) for r, v in t.items()}
        assert med["auto"] <= 1.10 * min(med["gpu"], med["cpu"]), (k, med, m)
    buf.close()


@pytest.mark.parametrize("layout", ["pinned", "pageable", "file"])
def test_route_split_vs_oracle(torch_cuda, oracle, tmp_path, layout):
    """S3H_ROUTE_SPLIT: the longest parts on the CPU drop-in while the GPU host path hashes the
    rest, at once -- ragged parts (empty, a few bytes, up to 6 MiB, in shuffled order),
    pinned, pageable and file ranges: every digest vs the oracle, the route reported, and the
    CPU side's share the model's plan (s3h_route_split_estimate).  One part is not split."""
    torch = torch_cuda
    rng = np.random.default_rng(4242 + len(layout))
    n = 600
    lens = rng.integers(0, 6 << 20, n).astype(np.uint64)
    lens[:5] = [0, 1, 63, 64, 0]
    lens = lens[rng.permutation(n)]
    offs = np.concatenate([[0], np.cumsum(lens + 7)[:-1]]).astype(np.uint64)
    total = int(offs[-1] + lens[-1]) + 64
    src = rng.integers(0, 256, total, dtype=np.uint8)
    want = oracle.batch(src, offs, lens, threads=16)
    k, _, _ = s3.route_split_estimate(lens, s3.route_model(), source=layout)
    assert 0 < k < n
    if layout == "file":
        path = tmp_path / "split.bin"
        src.tofile(path)
        got, taken = s3.sha256_file_parts_routed(str(path), offs, lens, route="split")
        one, taken1 = s3.sha256_file_parts_routed(str(path), offs[:1], lens[:1], route="split")
    else:
        buf = torch.empty(total, dtype=torch.uint8, pin_memory=layout == "pinned")
        buf.numpy()[:] = src
        got, taken = s3.sha256_batch_routed(s3.BufferParts(buf, offs, lens), route="split")
        one, taken1 = s3.sha256_batch_routed(s3.BufferParts(buf, offs[:1], lens[:1]), route="split")
    assert taken == "split" and taken1 == "gpu"
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, (layout, bad[:8])
    assert np.array_equal(one, want[:1])


@pytest.mark.parametrize("kind", ["pinned", "pageable"])
def test_verify_routed(torch_cuda, oracle, kind):
    """Download-side verification on every route (s3h_verify_batch_routed): ragged parts, about
    3 % of the expected digests corrupted in one bit; the mismatch mask is exactly the
    corrupted set on gpu / cpu / split / auto, for SHA-256 and (round 6) MD5 alike."""
    torch = torch_cuda
    rng = np.random.default_rng(77 + len(kind))
    n = 700
    lens = rng.integers(0, 2 << 20, n).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    total = int(lens.sum()) + 64
    src = rng.integers(0, 256, total, dtype=np.uint8)
    buf = torch.empty(total, dtype=torch.uint8, pin_memory=kind == "pinned")
    buf.numpy()[:] = src
    parts = s3.BufferParts(buf, offs, lens)
    exp = oracle.batch(src, offs, lens, threads=16).copy()
    bad = rng.random(n) < 0.03
    exp[bad, 3] ^= np.uint32(1 << 7)
    for route in ("gpu", "cpu", "split", "auto"):
        mask, taken = s3.verify_batch_routed(parts, exp, route=route)
        assert np.array_equal(mask, bad), route
        assert taken == route or route == "auto", (route, taken)
    m5 = oracle.md5_batch(src, offs, lens).copy()
    m5[bad, 0] ^= np.uint32(1)
    for route in ("gpu", "cpu", "split", "auto"):
        mask, taken = s3.verify_batch_routed(parts, m5, algo="md5", route=route)
        assert np.array_equal(mask, bad), route
        assert taken == route or route == "auto", (route, taken)


def test_concurrent_split_and_auto_callers(torch_cuda, oracle, tmp_path):
    """Six threads at once on the split and AUTO routes (each split starting its own CPU-side
    threads beside GPU sides that meet in the device queue): pinned and pageable parts, file
    ranges and a one-part batch, three rounds each; every digest vs the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(606)
    n = 400
    lens = rng.integers(0, 3 << 20, n).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    total = int(lens.sum()) + 64
    src = rng.integers(0, 256, total, dtype=np.uint8)
    want = oracle.batch(src, offs, lens, threads=16)
    pinned = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = src
    path = tmp_path / "split.bin"
    src.tofile(path)
    cases = [("split", "pinned"), ("auto", "pinned"), ("split", "pageable"), ("auto", "pageable"),
             ("split", "file"), ("split", "one")]
    errors, bad = [], []

    def job(k):
        route, kind = cases[k]
        sel = slice(k * 7, k * 7 + (1 if kind == "one" else n - 6 * 7))
        o, ln = offs[sel], lens[sel]
        try:
            for _ in range(3):
                if kind == "file":
                    got, _ = s3.sha256_file_parts_routed(str(path), o, ln, route=route)
                else:
                    buf = pinned if kind == "pinned" else src
                    got, _ = s3.sha256_batch_routed(s3.BufferParts(buf, o, ln), route=route)
                if not np.array_equal(got, want[sel]):
                    bad.append((route, kind))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=job, args=(k,)) for k in range(len(cases))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    assert not bad, bad


def test_dual_digest_host_beyond_one_grid(torch_cuda, oracle):
    """SHA-256 + MD5 from host memory for more parts than any one-grid dual form holds (9,000
    ragged pageable parts: the two plans per slice on the two hash streams) and, in another
    call, pinned parts of one length at a constant stride (2-D copies, tail-ramp slices): every
    digest of both algorithms vs the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(9000)
    n = 9000
    lens = rng.integers(0, 40000, n)
    lens[:4] = [0, 1, 55, 64]
    base = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    views = [base[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]
    sha, m5 = s3.sha256_md5_batch_host(views)
    assert np.array_equal(sha, oracle.batch(base, offs, lens, threads=16))
    assert np.array_equal(m5, oracle.md5_batch(base, offs, lens, threads=16))
    L, stride = 300_000, 300_032
    pinned = torch.empty(n * stride, dtype=torch.uint8, pin_memory=True)
    h = pinned.numpy()
    h[:] = rng.integers(0, 256, h.size, dtype=np.uint8)
    po = np.arange(n) * stride
    pv = [h[int(o):int(o) + L] for o in po]
    sha, m5 = s3.sha256_md5_batch_host(pv)
    pl = np.full(n, L)
    assert np.array_equal(sha, oracle.batch(h, po, pl, threads=16))
    assert np.array_equal(m5, oracle.md5_batch(h, po, pl, threads=16))
    del pinned, h, pv


def test_buffer_parts_match_views(torch_cuda, oracle):
    """BufferParts (pointers formed in numpy from one buffer) and a list of views give the
    same digests through every host entry point: SHA-256, MD5, both, verification and the
    routed call; pinned and pageable buffers; empty parts included."""
    torch = torch_cuda
    rng = np.random.default_rng(4242)
    n = 3000
    lens = rng.integers(0, 200000, n)
    lens[:4] = [0, 1, 64, 0]
    offs = np.concatenate([[0], np.cumsum(lens + 5)[:-1]])
    size = int(offs[-1] + lens[-1]) + 64
    pinned = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    for buf in (pinned, rng.integers(0, 256, size, dtype=np.uint8)):
        h = buf.numpy() if hasattr(buf, "numpy") else buf
        if hasattr(buf, "numpy"):
            h[:] = rng.integers(0, 256, size, dtype=np.uint8)
        bp = s3.BufferParts(buf, offs, lens)
        want = oracle.batch(h, offs, lens, threads=16)
        assert np.array_equal(s3.sha256_batch_host(bp), want)
        assert np.array_equal(s3.md5_batch_host(bp), oracle.md5_batch(h, offs, lens, threads=16))
        sha, m5 = s3.sha256_md5_batch_host(bp)
        assert np.array_equal(sha, want)
        exp = want.copy()
        exp[[7, 2999]] ^= 1
        assert np.flatnonzero(s3.verify_batch_host(bp, exp)).tolist() == [7, 2999]
        got, taken = s3.sha256_batch_routed(bp, route="gpu")
        assert np.array_equal(got, want) and taken == "gpu"
    del pinned


@pytest.mark.parametrize("layout", ["pinned_range", "pinned_shuffled", "pageable", "file", "dual",
                                    "pageable_mixed", "pinned_mixed"])
def test_many_small_parts_in_groups(torch_cuda, oracle, tmp_path, layout):
    """Thousands of small ragged parts (0 - 128 KiB, ~300 MiB: several groups of whole parts,
    run_host_groups) instead of slices of every part: pinned parts that are one increasing
    range of a buffer (DMA'd as the range), pinned parts in shuffled order (packed by the copy
    threads), pageable parts, file ranges (pread) and both digests at once; `mixed`: a few
    large parts (2 - 24 MiB) among them go through the slice pipeline afterwards.  Every
    digest vs the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(808 + len(layout))
    n = 4000
    lens = rng.integers(0, 128 << 10, n).astype(np.uint64)
    lens[rng.integers(0, n, 20)] = 0
    if layout.endswith("_mixed"):
        lens[rng.integers(0, n, 5)] = rng.integers(2 << 20, 24 << 20, 5)
        layout = layout[:-len("_mixed")]
    gaps = rng.integers(0, 16, n).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens + gaps)[:-1]]).astype(np.uint64)
    total = int(offs[-1] + lens[-1]) + 64
    src = rng.integers(0, 256, total, dtype=np.uint8)
    want = oracle.batch(src, offs, lens, threads=16)
    if layout == "file":
        path = tmp_path / "small.bin"
        src.tofile(path)
        got = s3.sha256_file_parts(str(path), offs, lens)
    else:
        buf = torch.empty(total, dtype=torch.uint8, pin_memory=layout.startswith("pinned") or layout == "dual")
        buf.numpy()[:] = src
        if layout == "pinned_shuffled":
            perm = rng.permutation(n)
            got = np.empty_like(want)
            got[perm] = s3.sha256_batch_host(s3.BufferParts(buf, offs[perm], lens[perm]))
        elif layout == "dual":
            got, m5 = s3.sha256_md5_batch_host(s3.BufferParts(buf, offs, lens))
            assert np.array_equal(m5, oracle.md5_batch(src, offs, lens))
        else:
            got = s3.sha256_batch_host(s3.BufferParts(buf, offs, lens))
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, (layout, bad[:8])


def test_group_dma_spans_one_pinned_allocation(torch_cuda, oracle, tmp_path):
    """Advisor r5 (high): many small pinned parts that form one increasing address range are
    DMA'd as that range -- only when the range lies inside ONE pinned allocation.  Parts taken
    from 120 separately pinned buffers, passed in increasing address order, have unregistered
    pages (or other allocations) between them: they must be packed like pageable parts, and
    every digest must equal the oracle's.  The same parts inside one pinned buffer still go as
    one range (S3H_TRACE_HOST reports which, in a child process)."""
    import subprocess
    import sys
    torch = torch_cuda
    rng = np.random.default_rng(911)
    n = 120
    lens = rng.integers(1, 60000, n)
    bufs = [s3.PinnedBuffer(int(L) + 4096) for L in lens]
    order = sorted(range(n), key=lambda i: bufs[i].ptr)
    views = []
    for i in order:
        a = bufs[i].array[:int(lens[i])]
        a[:] = rng.integers(0, 256, a.size, dtype=np.uint8)
        views.append(a)
    want = np.stack([oracle.sha256(v.tobytes()) for v in views])
    got = s3.sha256_batch_host(views)
    assert np.array_equal(got, want)
    sha, m5 = s3.sha256_md5_batch_host(views)
    assert np.array_equal(sha, want)
    assert np.array_equal(m5, np.stack([oracle.md5(v.tobytes()) for v in views]))
    code = f"""
import sys; sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
import numpy as np, torch, s3client_amd as s3
rng = np.random.default_rng(5)
n = 120
lens = rng.integers(1, 60000, n)
bufs = [s3.PinnedBuffer(int(L) + 4096) for L in lens]
order = sorted(range(n), key=lambda i: bufs[i].ptr)
apart = [bufs[i].array[:int(lens[i])] for i in order]
pad = (lens + 63) // 64 * 64  # packed at 64-B boundaries: the range spans the group's bytes
one = torch.empty(int(pad.sum()) + 64, dtype=torch.uint8, pin_memory=True)
offs = np.concatenate([[0], np.cumsum(pad)[:-1]])
s3.sha256_batch_host(apart)
s3.sha256_batch_host(s3.BufferParts(one, offs, lens))
print("ok")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "S3H_TRACE_HOST": "1"})
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]
    groups = [l for l in r.stderr.splitlines() if "groups of" in l]
    assert len(groups) == 2, r.stderr[-3000:]
    assert groups[0].endswith("(staged)"), groups  # separate allocations: packed
    assert groups[1].endswith("(pinned ranges)"), groups  # one buffer: one DMA per group
