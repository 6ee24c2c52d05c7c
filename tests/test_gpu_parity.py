"""GPU parity: the HIP kernels (through the C-ABI) against the oracle and the golden vectors.

Bar: bit-exact digests (integer work).  Sizes are chosen so the CPU oracle finishes in
seconds; the full C2 batch (1024 x 8 MiB) is checked part-by-part against the oracle too."""
import os

import numpy as np
import pytest

import s3client_amd as s3

from .kernel_choice import shared_range_kernel

pytestmark = pytest.mark.gpu
SEED = 20241008
KERNELS = ["skew", "skewp", "skews", "quad", "pair", "pc", "lane"]


def _dev_buffer(torch, host: np.ndarray):
    t = torch.empty(max(host.size, 1), dtype=torch.uint8, device="cuda")
    if host.size:
        t.copy_(torch.from_numpy(host))
    return t


def _run(torch, host_buf, offs, lens, kernel):
    data = _dev_buffer(torch, host_buf)
    out = s3.sha256_batch_device(data, offs, lens, kernel=kernel)
    return out.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("kernel", KERNELS)
def test_length_edges_all_alignments(torch_cuda, oracle, golden, kernel):
    """Every golden edge length, placed at byte misalignments 0..3 and 13 (v_perm decode)."""
    edges = [e for e in golden["edge"] if e["L"] <= (1 << 20) + 13]
    big = np.frombuffer(oracle.generate(7, max(e["L"] for e in edges)), dtype=np.uint8)
    offs, lens, want, chunks, pos = [], [], [], [], 0
    for mis in (0, 1, 2, 3, 13):
        for e in edges:
            pos += (-pos) % 64 + mis
            offs.append(pos)
            lens.append(e["L"])
            want.append(e["digest"])
            chunks.append((pos, big[:e["L"]]))
            pos += e["L"]
    host = np.zeros(pos + 64, dtype=np.uint8)
    for o, c in chunks:
        host[o:o + c.size] = c
    got = s3.digests_to_text(_run(torch_cuda, host, offs, lens, kernel))
    bad = [(lens[i], offs[i] % 4) for i in range(len(want)) if got[i] != want[i]]
    assert not bad, bad[:10]


@pytest.mark.parametrize("kernel", KERNELS)
def test_random_ragged_vs_oracle(torch_cuda, oracle, kernel):
    rng = np.random.default_rng(2024)
    n = 777
    lens = rng.integers(0, 20000, n)
    lens[:5] = [0, 0, 55, 56, 64]  # empty parts and padding edges
    gaps = rng.integers(0, 100, n)
    offs = np.cumsum(gaps + np.concatenate([[0], lens[:-1]]))
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 8, dtype=np.uint8)
    got = _run(torch_cuda, host, offs, lens, kernel)
    want = oracle.batch(host, offs, lens)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("kernel", ["skews", "skew"])
def test_constant_byte_parts(torch_cuda, kernel):
    """Constant-byte parts (0x00, 0x01, 0x7f, 0x80, 0xff, 0xa5) at misalignments 0 and 3: the
    extremes of the shared-SIMD producer's denormal v_mul_f32 left shifts (tools/gen_producer.py
    mulf_ok), checked against hashlib."""
    import hashlib
    fills, lens = (0x00, 0x01, 0x7F, 0x80, 0xFF, 0xA5), (64, 1000, 65536 + 55, (1 << 20) + 13)
    offs, want, pos, chunks = [], [], 0, []
    for mis in (0, 3):
        for f in fills:
            for L in lens:
                pos += (-pos) % 64 + mis
                offs.append(pos)
                chunks.append((pos, L, f))
                want.append(hashlib.sha256(bytes([f]) * L).hexdigest())
                pos += L
    host = np.zeros(pos + 64, dtype=np.uint8)
    for o, L, f in chunks:
        host[o:o + L] = f
    got = s3.digests_to_text(_run(torch_cuda, host, offs, [c[1] for c in chunks], kernel))
    bad = [(c[2], c[1], c[0] % 4) for c, g, w in zip(chunks, got, want) if g != w]
    assert not bad, bad[:10]


def test_kernels_agree_on_many_small_parts(torch_cuda, oracle):
    """n > 65536 exercises the AUTO switch to the fused kernel; overlapping parts allowed."""
    assert s3.Plan([0] * 70000, [1] * 70000).info()["kernel"] == "lane"
    assert s3.Plan([0] * 40000, [1] * 40000).info()["kernel"] == "pc"
    assert s3.Plan([0] * 1024, [1] * 1024).info()["kernel"] == "skew"
    assert s3.Plan([0] * 10000, [1] * 10000).info()["kernel"] == "skewp"
    assert s3.Plan([0] * 8192, [1] * 8192).info()["kernel"] == shared_range_kernel()
    assert s3.Plan([0] * 4097, [1] * 4097).info()["kernel"] == shared_range_kernel()
    assert s3.Plan([0] * 30000, [1] * 30000).info()["kernel"] == "pair"
    rng = np.random.default_rng(7)
    n = 70000
    lens = rng.integers(0, 200, n)
    offs = rng.integers(0, 1 << 20, n)
    host = rng.integers(0, 256, (1 << 20) + 256, dtype=np.uint8)
    data = _dev_buffer(torch_cuda, host)
    a = s3.sha256_batch_device(data, offs, lens, kernel="auto").cpu().numpy().view(np.uint32)
    for k in ("pc", "pair", "quad", "skew", "skewp", "skews"):
        b = s3.sha256_batch_device(data, offs, lens, kernel=k).cpu().numpy().view(np.uint32)
        assert np.array_equal(a, b), k
    idx = rng.choice(n, 500, replace=False)
    want = oracle.batch(host, offs[idx], lens[idx])
    assert np.array_equal(a[idx], want)


def test_device_generator_matches_oracle(torch_cuda, oracle):
    lens = [0, 1, 7, 8, 9, 1000, 4097, 65536 + 3]
    offs = np.concatenate([[0], np.cumsum([(L + 255) // 256 * 256 for L in lens])[:-1]])
    ids = [5, 6, 7, 8, 9, 10, 11, 1023]
    data = torch_cuda.zeros(int(offs[-1] + lens[-1]) + 256, dtype=torch_cuda.uint8, device="cuda")
    s3.generate_parts(data, offs, lens, ids, SEED)
    host = data.cpu().numpy()
    for o, L, p in zip(offs, lens, ids):
        assert host[o:o + L].tobytes() == oracle.generate(p, L), (p, L)


def _c2(torch, nparts):
    L = 8 << 20
    offs = np.arange(nparts, dtype=np.uint64) * L
    lens = np.full(nparts, L, dtype=np.uint64)
    data = torch.empty(nparts * L, dtype=torch.uint8, device="cuda")
    s3.generate_parts(data, offs, lens, np.arange(nparts), SEED)
    return data, offs, lens


@pytest.fixture(scope="module")
def c2_batch(torch_cuda, oracle):
    """BASELINE config 2 in HBM (1024 x 8 MiB) and the oracle's 1024 digests of the same bytes."""
    data, offs, lens = _c2(torch_cuda, 1024)
    want = oracle.batch(data.cpu().numpy(), offs, lens, threads=16)
    yield data, offs, lens, want
    del data
    torch_cuda.cuda.empty_cache()


@pytest.mark.parametrize("kernel", KERNELS)
def test_c2_full_batch_bit_exact(torch_cuda, golden, c2_batch, kernel):
    """BASELINE config 2: 1024 x 8 MiB in HBM; fixtures p in {0..15, 511, 1022, 1023} and all
    1024 digests against the oracle on the same bytes, for every kernel."""
    data, offs, lens, want = c2_batch
    out = s3.sha256_batch_device(data, offs, lens, kernel=kernel).cpu().numpy().view(np.uint32)
    txt = s3.digests_to_text(out)
    for e in golden["c2_parts"]:
        assert txt[e["p"]] == e["digest"], e["p"]
    assert np.array_equal(out, want)


def test_resumable_ranges_match_single_launch(torch_cuda, oracle):
    rng = np.random.default_rng(11)
    n = 200
    lens = rng.integers(0, 300000, n)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    host = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    data = _dev_buffer(torch_cuda, host)
    for kernel in KERNELS:
        plan = s3.Plan(offs, lens, kernel=kernel)
        one = torch_cuda.zeros((n, 8), dtype=torch_cuda.int32, device="cuda")
        plan.launch(data, one)
        many = torch_cuda.zeros((n, 8), dtype=torch_cuda.int32, device="cuda")
        mb = plan.info()["max_blocks"]
        step = 977
        for b0 in range(0, mb, step):
            plan.launch_range(data.data_ptr(), many, b0, b0 + step, 0)
        torch_cuda.cuda.synchronize()
        assert torch_cuda.equal(one, many), kernel
        assert np.array_equal(one.cpu().numpy().view(np.uint32), oracle.batch(host, offs, lens))
        plan.close()


def test_host_path_transfer_geometry(torch_cuda, golden):
    """test/parallel-file-transfer-test.cpp data sliced by lib/src/upload.cpp geometry, hashed
    from HOST memory (H2D included), against the reference's digests."""
    t = golden["transfer"]
    data = (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8)
    parts = s3.upload_parts_geometry(t["size"], t["jobs"], t["parts_per_job"])
    assert [(p.offset, p.size) for p in parts] == [(q["offset"], q["size"]) for q in t["parts"]]
    from s3client_amd.upload import payload_hashes
    assert payload_hashes(data, parts) == [q["digest"] for q in t["parts"]]


def test_host_path_multipart_and_small_slices(torch_cuda, golden):
    mp = golden["multipart"]
    data = (np.arange(mp["size"], dtype=np.uint64) % 256).astype(np.uint8)
    views = [data[p["offset"]:p["offset"] + p["size"]] for p in mp["parts"]]
    for sl in (0, 64, 4096 * 3, 1 << 20):
        got = s3.digests_to_text(s3.sha256_batch_host(views, slice_bytes=sl))
        assert got == [p["digest"] for p in mp["parts"]], sl


def test_c3_parts_ragged(torch_cuda, oracle, golden):
    """The whole BASELINE config-3 parts that have lib/hash fixtures (5.0-64 MiB, not
    multiples of 64) as one small batch, plus a ragged batch of 64 C3-distributed lengths
    scaled down 64x, packed at 256-B offsets, on every kernel."""
    lens = [e["L"] for e in golden["c3_parts"]]
    offs = np.concatenate([[0], np.cumsum([(L + 255) // 256 * 256 for L in lens])[:-1]])
    data = torch_cuda.empty(int(offs[-1]) + lens[-1] + 256, dtype=torch_cuda.uint8, device="cuda")
    s3.generate_parts(data, offs, lens, [e["p"] for e in golden["c3_parts"]], SEED)
    got = s3.digests_to_text(s3.sha256_batch_device(data, offs, lens).cpu().numpy())
    assert got == [e["digest"] for e in golden["c3_parts"]]
    small = [L // 64 + 3 for L in golden["c3_lengths"]]
    so = np.concatenate([[0], np.cumsum([(L + 255) // 256 * 256 for L in small])[:-1]])
    d2 = torch_cuda.empty(int(so[-1]) + small[-1] + 256, dtype=torch_cuda.uint8, device="cuda")
    s3.generate_parts(d2, so, small, range(64), SEED)
    for k in KERNELS:
        g2 = s3.sha256_batch_device(d2, so, small, kernel=k).cpu().numpy().view(np.uint32)
        assert np.array_equal(g2, oracle.batch(d2.cpu().numpy(), so, small)), k


def test_plan_rejects_undersized_buffers(torch_cuda):
    data = torch_cuda.empty(100, dtype=torch_cuda.uint8, device="cuda")
    dig = torch_cuda.empty((1, 8), dtype=torch_cuda.int32, device="cuda")
    plan = s3.Plan([50], [60])
    with pytest.raises(ValueError):
        plan.launch(data, dig)


def test_host_path_small_slices_large_batch(torch_cuda, oracle):
    """Host streaming with many slices per part: every ranged launch must load only bytes of
    its own slice (regression: prefetches once ran one block past the ring slot)."""
    rng = np.random.default_rng(3)
    lens = [2 << 20, (2 << 20) + 13, 1 << 20, 777777, 0, 64, 300000] * 20
    parts = [rng.integers(0, 256, L, dtype=np.uint8) for L in lens]
    want = np.stack([oracle.sha256(p.tobytes()) for p in parts])
    for sl in (256 << 10, 64 << 10):
        assert np.array_equal(s3.sha256_batch_host(parts, slice_bytes=sl), want), sl


def test_host_path_uniform_stride_2d_copies(torch_cuda, oracle):
    """Equal-length parts at a constant host stride take the one-2D-copy-per-slice path."""
    rng = np.random.default_rng(4)
    L, stride, n = (1 << 20) + 7, (1 << 20) + 64, 64
    buf = rng.integers(0, 256, stride * n, dtype=np.uint8)
    views = [buf[i * stride:i * stride + L] for i in range(n)]
    want = oracle.batch(buf, np.arange(n) * stride, np.full(n, L))
    for sl in (64 << 10, 256 << 10, 0):
        assert np.array_equal(s3.sha256_batch_host(views, slice_bytes=sl), want), sl


# ------------------------------------------------------------------ MD5
def test_md5_edges_all_alignments(torch_cuda, oracle, golden):
    md = golden["md5"]
    edges = [e for e in md["edge"] if e["L"] <= (1 << 20) + 13]
    big = np.frombuffer(oracle.generate(7, max(e["L"] for e in edges)), dtype=np.uint8)
    offs, lens, want, chunks, pos = [], [], [], [], 0
    for mis in (0, 1, 2, 3, 13):
        for e in edges:
            pos += (-pos) % 64 + mis
            offs.append(pos); lens.append(e["L"]); want.append(e["digest"])
            chunks.append((pos, big[:e["L"]]))
            pos += e["L"]
    host = np.zeros(pos + 64, dtype=np.uint8)
    for o, c in chunks:
        host[o:o + c.size] = c
    data = _dev_buffer(torch_cuda, host)
    got = s3.digests_to_text(s3.md5_batch_device(data, offs, lens).cpu().numpy(), 4)
    assert got == want


def test_md5_c2_and_ragged_vs_oracle(torch_cuda, oracle, golden, c2_batch):
    data, offs, lens, _ = c2_batch
    out = s3.md5_batch_device(data, offs, lens).cpu().numpy().view(np.uint32)
    txt = s3.digests_to_text(out, 4)
    for e in golden["md5"]["c2_parts"]:
        assert txt[e["p"]] == e["digest"], e["p"]
    assert np.array_equal(out, oracle.md5_batch(data.cpu().numpy(), offs, lens, threads=16))
    rng = np.random.default_rng(21)
    n = 500
    rl = rng.integers(0, 30000, n)
    ro = np.cumsum(rng.integers(0, 50, n) + np.concatenate([[0], rl[:-1]]))
    host = rng.integers(0, 256, int(ro[-1] + rl[-1]) + 8, dtype=np.uint8)
    got = s3.md5_batch_device(_dev_buffer(torch_cuda, host), ro, rl).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, oracle.md5_batch(host, ro, rl))


def test_md5_host_path_transfer_etag(torch_cuda, golden):
    t = golden["transfer"]
    data = (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8)
    views = [data[p["offset"]:p["offset"] + p["size"]] for p in t["parts"]]
    for sl in (0, 64 << 10):
        d = s3.md5_batch_host(views, slice_bytes=sl)
        assert s3.digests_to_text(d, 4) == [p["digest"] for p in golden["md5"]["transfer"]]
        assert s3.multipart_etag(d) == golden["md5"]["transfer_etag"]


def test_md5_beyond_one_workgroup_per_cu(torch_cuda, oracle):
    """MD5 batches whose grid has more workgroups than the GPU has CUs (> 64 x CUs parts: 20,000
    here) run md5_pc_kernel<1> (1-block steps, 32 KiB of LDS, several workgroups per CU;
    capi.hip launch): ragged, misaligned parts incl. empty ones, device-resident and through
    the host path with slices of an odd number of blocks, bit-exact vs the oracle."""
    rng = np.random.default_rng(2020)
    n = 20000
    lens = rng.integers(0, 40000, n)
    lens[:6] = [0, 1, 55, 56, 64, 119]
    offs = np.concatenate([[0], np.cumsum(lens + rng.integers(0, 9, n))[:-1]])
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    cus = torch_cuda.cuda.get_device_properties(0).multi_processor_count
    with s3.Plan(offs, lens, algo="md5") as plan:
        assert plan.info()["grid"] == (n + 63) // 64 > cus
    want = oracle.md5_batch(host, offs, lens, threads=16)
    got = s3.md5_batch_device(_dev_buffer(torch_cuda, host), offs, lens).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)
    views = [host[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]
    for sl in (37 * 64, 101 * 64, 0):
        assert np.array_equal(s3.md5_batch_host(views, slice_bytes=sl), want), sl


@pytest.mark.parametrize("n,shape,apart", [(2100, "ragged", True), (3000, "ragged", True),
                                           (5500, "ragged", False), (2100, "between", False)])
def test_dual_mixed_grid_ragged(torch_cuda, oracle, n, shape, apart):
    """SHA-256 + MD5 of a ragged batch in the skewp-group range (C3-like lengths, scaled):
    the one-grid mixed kernel (the longest parts in skew groups, the rest in skewp groups,
    slot arrays offset for the second half) vs the oracle, device- and host-resident, BOTH
    forms of it: the skew groups' MD5 on workgroups of their own (2,100 / 3,000 parts) and,
    when that grid would exceed one workgroup per CU (5,500 parts), inside each skew group.
    "between": one longest part and 2,099 at 0.85 of it -- every part needs a skew group at
    the apart form's rate ratio, so only the in-group form's smaller ratio gives a mixed grid
    (F = 1; before the advisor-r4 fix this fell to the plain group kernel).  Equal lengths keep
    the plain group kernel (dual_solo 0)."""
    rng = np.random.default_rng(n)
    if shape == "between":
        lens = np.full(n, int(64 * 1024 * 0.85), dtype=np.int64)
        lens[0] = 64 * 1024
    else:
        lens = 5 * 1024 + rng.integers(0, 59 * 1024 + 1, n)
        lens[:5] = [64 * 1024, 64 * 1024 - 1, 0, 55, 64 * 1024 + 9]
    offs = np.concatenate([[0], np.cumsum(lens + 7)[:-1]])
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    with s3.Plan(offs, lens) as plan:
        info = plan.info()
    solo = info["dual_solo"]
    assert 0 < solo and 8 * solo < n
    assert info["dual_apart"] == apart
    assert s3.dual_layout(lens, torch_cuda.cuda.get_device_properties(0).multi_processor_count) == (solo, apart)
    if shape == "between":
        assert solo == 1
    data = _dev_buffer(torch_cuda, host)
    sha, m5 = s3.sha256_md5_batch_device(data, offs, lens)
    want_sha, want_md5 = oracle.batch(host, offs, lens), oracle.md5_batch(host, offs, lens)
    assert np.array_equal(sha.cpu().numpy().view(np.uint32), want_sha)
    assert np.array_equal(m5.cpu().numpy().view(np.uint32), want_md5)
    views = [host[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]
    hsha, hm5 = s3.sha256_md5_batch_host(views)
    assert np.array_equal(hsha, want_sha) and np.array_equal(hm5, want_md5)
    eq = np.full(n, 20000, dtype=np.uint64)
    with s3.Plan(np.arange(n, dtype=np.uint64) * 20000, eq) as plan:
        assert plan.info()["dual_solo"] == 0


@pytest.mark.parametrize("slice_blocks", [5, 7, 9])
def test_md5_odd_slices_mix_full_and_partial_steps(torch_cuda, oracle, slice_blocks):
    """Host path with slices of an odd number of 64-B blocks: every resumable launch starts
    mid-part at a block offset that is not a multiple of the 4-block producer step, so each
    one runs full steps through the rolling fused statement and a partial step through the
    checked per-block path, the chaining state carried between launches (MD5 alone and both
    digests), vs the oracle."""
    rng = np.random.default_rng(slice_blocks)
    lens = rng.integers(0, 5000, 90)
    lens[:3] = [0, 64 * slice_blocks, 64 * slice_blocks * 3 + 55]
    parts = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in lens]
    want = np.stack([oracle.md5(p.tobytes()) for p in parts])
    got = s3.md5_batch_host(parts, slice_bytes=64 * slice_blocks)
    assert np.array_equal(got, want)
    sha, m5 = s3.sha256_md5_batch_host(parts, slice_bytes=64 * slice_blocks)
    assert np.array_equal(m5, want)
    assert np.array_equal(sha, np.stack([oracle.sha256(p.tobytes()) for p in parts]))


def test_verify_download_parts(torch_cuda, golden):
    """Download-side verification: one corrupted byte flags exactly its part."""
    t = golden["transfer"]
    data = (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8)
    views = [data[p["offset"]:p["offset"] + p["size"]].copy() for p in t["parts"]]
    views[4][12345] ^= 1
    sha = [p["digest"] for p in t["parts"]]
    md5s = [p["digest"] for p in golden["md5"]["transfer"]]
    assert s3.verify_batch_host(views, sha).tolist() == [False] * 4 + [True, False]
    assert s3.verify_batch_host(views, md5s, algo="md5").tolist() == [False] * 4 + [True, False]
    dev = torch_cuda.from_numpy(np.concatenate(views)).cuda()
    offs = np.concatenate([[0], np.cumsum([v.size for v in views])[:-1]])
    exp = torch_cuda.from_numpy(np.stack([np.frombuffer(bytes.fromhex(h), np.uint32)
                                          for h in sha]).view(np.int32)).cuda()
    n, mask = s3.verify_batch_device(dev, offs, [v.size for v in views], exp)
    assert n == 1 and mask.cpu().tolist() == [False] * 4 + [True, False]


@pytest.mark.parametrize("kernel", ["quad", "skew"])
def test_quad_two_consumer_waves_ragged(torch_cuda, oracle, kernel):
    """3,000 parts: the quad / skew plan runs two consumer waves per workgroup (grid 188)."""
    rng = np.random.default_rng(31)
    n = 3000
    plan = s3.Plan([0] * n, [1] * n, kernel=kernel)
    assert plan.info()["grid"] == (n + 15) // 16
    lens = rng.integers(0, 9000, n)
    lens[:4] = [0, 55, 56, 64]
    offs = np.concatenate([[0], np.cumsum(lens + rng.integers(0, 5, n))[:-1]])
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 8, dtype=np.uint8)
    got = _run(torch_cuda, host, offs, lens, kernel)
    assert np.array_equal(got, oracle.batch(host, offs, lens))


# ------------------------------------------------------------------ dual digest (SHA-256 + MD5)
def test_dual_digest_host_transfer_and_ragged(torch_cuda, oracle, golden):
    """s3h_sha256_md5_batch_host: one H2D pass, both digests bit-exact (reference transfer
    parts: SHA-256 goldens, MD5 goldens + ETag; ragged random parts vs the oracle)."""
    t = golden["transfer"]
    data = (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8)
    views = [data[p["offset"]:p["offset"] + p["size"]] for p in t["parts"]]
    for sl in (0, 64 << 10):
        sha, m5 = s3.sha256_md5_batch_host(views, slice_bytes=sl)
        assert s3.digests_to_text(sha) == [p["digest"] for p in t["parts"]]
        assert s3.digests_to_text(m5, 4) == [p["digest"] for p in golden["md5"]["transfer"]]
        assert s3.multipart_etag(m5) == golden["md5"]["transfer_etag"]
    rng = np.random.default_rng(31)
    lens = [0, 1, 55, 56, 63, 64, 65, 119, 4087, 4088, 300001, (1 << 20) + 13] * 6
    parts = [rng.integers(0, 256, L, dtype=np.uint8) for L in lens]
    sha, m5 = s3.sha256_md5_batch_host(parts, slice_bytes=64 << 10)
    assert np.array_equal(sha, np.stack([oracle.sha256(p.tobytes()) for p in parts]))
    assert np.array_equal(m5, np.stack([oracle.md5(p.tobytes()) for p in parts]))


def test_dual_digest_device_c2_subset(torch_cuda, oracle, golden):
    """s3h_sha256_md5_batch_device on C2 parts: SHA-256 and MD5 goldens, and every part vs
    the single-algorithm batch entry points."""
    data, offs, lens = _c2(torch_cuda, 256)
    sha, m5 = s3.sha256_md5_batch_device(data, offs, lens)
    sha = sha.cpu().numpy().view(np.uint32)
    m5 = m5.cpu().numpy().view(np.uint32)
    txt = s3.digests_to_text(sha)
    for e in golden["c2_parts"]:
        if e["p"] < 256:
            assert txt[e["p"]] == e["digest"], e["p"]
    m5txt = s3.digests_to_text(m5, 4)
    for e in golden["md5"]["c2_parts"]:
        if e["p"] < 256:
            assert m5txt[e["p"]] == e["digest"], e["p"]
    assert np.array_equal(sha, s3.sha256_batch_device(data, offs, lens).cpu().numpy().view(np.uint32))
    assert np.array_equal(m5, s3.md5_batch_device(data, offs, lens).cpu().numpy().view(np.uint32))


def test_dual_digest_device_fallback_and_fused_ragged(torch_cuda, oracle):
    """Ragged batches on the dual-digest routes: 300 parts (split grid: skew workgroups then MD5
    workgroups), 2,000 parts (the split grid would not fit one workgroup per CU: skew groups
    each with a self-fed MD5 wave), 2,500 parts (two-group skew range: the group kernel's
    skewp geometry), and 9,000 / 33,000 parts (beyond every one-grid form: the SHA-256 and MD5
    kernels one after the other on the caller's stream -- skewp / pc with md5_pc_kernel<1>),
    each vs the oracle."""
    rng = np.random.default_rng(33)
    for n in (300, 2000, 2500, 9000, 33000):
        rl = rng.integers(0, 9000, n)
        ro = np.cumsum(rng.integers(0, 70, n) + np.concatenate([[0], rl[:-1]]))
        host = rng.integers(0, 256, int(ro[-1] + rl[-1]) + 8, dtype=np.uint8)
        sha, m5 = s3.sha256_md5_batch_device(_dev_buffer(torch_cuda, host), ro, rl)
        assert np.array_equal(sha.cpu().numpy().view(np.uint32), oracle.batch(host, ro, rl)), n
        assert np.array_equal(m5.cpu().numpy().view(np.uint32), oracle.md5_batch(host, ro, rl)), n


def test_host_path_pinned_and_pageable_agree(torch_cuda, oracle):
    """Pinned parts go straight to the copy engine; pageable ones through the pinned staging
    ring filled by host threads.  Same digests either way, oracle-exact."""
    rng = np.random.default_rng(41)
    lens = [0, 1, 64, 65, 5000, 70001, (1 << 20) + 3, 3 << 20] * 8
    total = sum(lens) + 64 * len(lens)
    pinned = torch_cuda.empty(total, dtype=torch_cuda.uint8, pin_memory=True)
    h = pinned.numpy()
    h[:] = rng.integers(0, 256, total, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(np.array(lens) + 64)[:-1]])
    views = [h[o:o + L] for o, L in zip(offs, lens)]
    copies = [v.copy() for v in views]  # pageable
    want = np.stack([oracle.sha256(v.tobytes()) for v in views])
    assert np.array_equal(s3.sha256_batch_host(views), want)
    assert np.array_equal(s3.sha256_batch_host(copies), want)
    sha, _ = s3.sha256_md5_batch_host(copies)
    assert np.array_equal(sha, want)


def test_dual_digest_group_kernel_device_and_host(torch_cuda, oracle):
    """sha256_md5_group_kernel (skewp SHA-256 group + MD5 group of the same 32 parts in one
    flag-synchronised workgroup): 8,192 ragged parts on the device (grid 256), and 5,000
    pageable host parts streamed in 4 KiB slices (ranged launches of the same kernel)."""
    rng = np.random.default_rng(61)
    n = 8192
    rl = rng.integers(0, 6000, n)
    rl[:4] = [0, 55, 56, 64]
    ro = np.cumsum(rng.integers(0, 40, n) + np.concatenate([[0], rl[:-1]]))
    host = rng.integers(0, 256, int(ro[-1] + rl[-1]) + 8, dtype=np.uint8)
    # SHA-256 alone: the shared-range kernel; both digests: the group kernel
    assert s3.Plan(ro, rl).info()["kernel"] == shared_range_kernel()
    sha, m5 = s3.sha256_md5_batch_device(_dev_buffer(torch_cuda, host), ro, rl)
    assert np.array_equal(sha.cpu().numpy().view(np.uint32), oracle.batch(host, ro, rl))
    assert np.array_equal(m5.cpu().numpy().view(np.uint32), oracle.md5_batch(host, ro, rl))
    parts = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 20000, 5000)]
    sha, m5 = s3.sha256_md5_batch_host(parts, slice_bytes=4096)
    assert np.array_equal(sha, np.stack([oracle.sha256(p.tobytes()) for p in parts]))
    assert np.array_equal(m5, np.stack([oracle.md5(p.tobytes()) for p in parts]))


@pytest.mark.parametrize("n,kernel", [(3000, "skew"), (5000, "skewp"), (5000, "skews")])
def test_flag_synchronised_kernels_resumable(torch_cuda, oracle, n, kernel):
    """The two-group skew kernel (2,049-4,096 parts) and skewp: resumable ranged launches of
    odd block counts == one launch == the oracle (the step counters restart per launch)."""
    rng = np.random.default_rng(62)
    lens = rng.integers(0, 40000, n)
    lens[:3] = [0, 63, 64]
    offs = np.concatenate([[0], np.cumsum(lens + 3)[:-1]])
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 8, dtype=np.uint8)
    data = _dev_buffer(torch_cuda, host)
    plan = s3.Plan(offs, lens, kernel=kernel)
    if kernel == "skew":  # two groups per workgroup except the solo ones (ragged batch)
        info = plan.info()
        g = (n + 7) // 8
        assert info["groups"] == g and info["grid"] == info["solo"] + (g - info["solo"] + 1) // 2
    one = torch_cuda.zeros((n, 8), dtype=torch_cuda.int32, device="cuda")
    plan.launch(data, one)
    many = torch_cuda.zeros((n, 8), dtype=torch_cuda.int32, device="cuda")
    for b0 in range(0, plan.info()["max_blocks"], 101):
        plan.launch_range(data.data_ptr(), many, b0, b0 + 101, 0)
    torch_cuda.cuda.synchronize()
    assert torch_cuda.equal(one, many)
    assert np.array_equal(one.cpu().numpy().view(np.uint32), oracle.batch(host, offs, lens))
    plan.close()


AUTO_EDGES = [(1, "skew"), (2048, "skew"), (2049, "skew"), (4096, "skew"), (4097, "skews"),
              (8192, "skews"), (8193, "skewp"), (28672, "skewp"), (28673, "pair"),
              (32768, "pair"), (32769, "pc"), (65536, "pc"), (65537, "lane")]


def test_auto_kernel_edges(torch_cuda, oracle):
    """Every AUTO switch point of plan.cpp resolve_kernel, one part below and above: the plan
    picks the documented kernel and every digest of ragged small parts (0-300 B,
    all byte alignments) matches the oracle; SHA-256 + MD5 from the dual path at the dual
    kernel's switch points (split grid / skew group / skewp group / two streams) vs the oracle
    as well."""
    rng = np.random.default_rng(62)
    host = rng.integers(0, 256, (1 << 20) + 512, dtype=np.uint8)
    data = _dev_buffer(torch_cuda, host)
    for n, kernel in AUTO_EDGES:
        lens = rng.integers(0, 300, n)
        offs = rng.integers(0, 1 << 20, n)
        want = shared_range_kernel() if kernel == "skews" else kernel  # default "power" policy
        assert s3.Plan(offs, lens).info()["kernel"] == want, n
        got = s3.sha256_batch_device(data, offs, lens).cpu().numpy().view(np.uint32)
        assert np.array_equal(got, oracle.batch(host, offs, lens, threads=16)), n
    for n in (1792, 1793, 1820, 2048, 2049, 4096, 4097, 8192, 8193):
        lens = rng.integers(0, 300, n)
        offs = rng.integers(0, 1 << 20, n)
        sha, m5 = s3.sha256_md5_batch_device(data, offs, lens)
        assert np.array_equal(sha.cpu().numpy().view(np.uint32),
                              oracle.batch(host, offs, lens, threads=16)), n
        assert np.array_equal(m5.cpu().numpy().view(np.uint32),
                              oracle.md5_batch(host, offs, lens, threads=16)), n
