"""BASELINE configs 3 and 4 at full size on one MI355X (pytest -m gpu).

C3 (configs[2]): 4096 parts of U[5,64] MiB (~138 GiB resident in HBM), AUTO -> the two-group
skew kernel with solo workgroups for the longest parts (grid > 256: capi.hip plan_solo).  C4 (configs[3]): rank 0's shard of 65,536 x 8 MiB over
8 GPUs -- global parts p = 8k, 8,192 x 8 MiB = 64 GiB -- AUTO -> skews (and skewp, compared).  Each batch is checked
against (i) the lib/hash golden digests of the parts that have fixtures (tests/golden: C3 ids
incl. the longest and shortest part, C4 ids of rank 0) and (ii) the oracle on EVERY part, the
device buffer copied back in <= 8 GiB chunks (C3: all 4,096 SHA-256 and MD5 digests of the
mixed dual grid too; the C4 shard: all 8,192, skews and skewp).  Bar: bit-exact."""
import numpy as np
import pytest

import s3client_amd as s3

from .kernel_choice import shared_range_kernel

pytestmark = pytest.mark.gpu
SEED = 20241008
MIB = 1 << 20


def _oracle_sample(torch, oracle, data, offs, lens, slots, threads=16):
    """Oracle digests of the parts in `slots`, copied out of the device buffer."""
    chunks = [data[int(offs[i]):int(offs[i]) + int(lens[i])].cpu().numpy() for i in slots]
    host = np.concatenate(chunks)
    so = np.concatenate([[0], np.cumsum([c.size for c in chunks])[:-1]]).astype(np.uint64)
    return oracle.batch(host, so, [c.size for c in chunks], threads=threads)


def _oracle_whole(torch, oracle, data, offs, lens, md5=False, chunk=8 << 30, threads=16):
    """Oracle digests of EVERY part of the device buffer (parts in ascending offset order):
    consecutive parts are copied back together through one pinned host buffer of at most
    `chunk` bytes and hashed by the oracle on `threads` threads.  -> (sha256, md5 or None)."""
    n = len(lens)
    offs = np.asarray(offs, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint64)
    assert np.all(np.diff(offs.astype(np.int64)) >= 0)
    ends = offs + lens
    assert int(lens.max()) <= chunk
    host = torch.empty(chunk, dtype=torch.uint8, pin_memory=True)
    sha = np.zeros((n, 8), dtype=np.uint32)
    m5 = np.zeros((n, 4), dtype=np.uint32) if md5 else None
    i = 0
    while i < n:
        j = i + 1
        while j < n and int(ends[j]) - int(offs[i]) <= chunk:
            j += 1
        a, b = int(offs[i]), int(ends[j - 1])
        host[:b - a].copy_(data[a:b])
        h = host.numpy()
        o = offs[i:j] - np.uint64(a)
        sha[i:j] = oracle.batch(h, o, lens[i:j], threads=threads)
        if md5:
            m5[i:j] = oracle.md5_batch(h, o, lens[i:j], threads=threads)
        i = j
    del host
    return sha, m5


def _hashlib_whole(torch, data, offs, lens, chunk=8 << 30, threads=16):
    """SHA-256 of EVERY part of the device buffer by Python's hashlib (OpenSSL: an independent
    implementation, pinned to lib/hash by the golden tests; it releases the GIL, so 16 threads
    hash in parallel) -- for the multi-shard checks whose volume (512 GiB for BASELINE config 4
    whole) the scalar oracle would take minutes over.  Same chunked pinned copy-back as
    _oracle_whole.  -> (n, 8) uint32."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    n = len(lens)
    offs = np.asarray(offs, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint64)
    ends = offs + lens
    host = torch.empty(chunk, dtype=torch.uint8, pin_memory=True)
    out = np.zeros((n, 8), dtype=np.uint32)
    with ThreadPoolExecutor(threads) as pool:
        i = 0
        while i < n:
            j = i + 1
            while j < n and int(ends[j]) - int(offs[i]) <= chunk:
                j += 1
            a, b = int(offs[i]), int(ends[j - 1])
            host[:b - a].copy_(data[a:b])
            mv = memoryview(host.numpy())

            def one(k, a=a, mv=mv):
                o = int(offs[k]) - a
                out[k] = np.frombuffer(hashlib.sha256(mv[o:o + int(lens[k])]).digest(), dtype=np.uint32)
            list(pool.map(one, range(i, j)))
            i = j
    del host
    return out


def _release(torch):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_c3_full_ragged_batch(torch_cuda, oracle, golden):
    torch = torch_cuda
    n = 4096
    lens = np.array([oracle.c3_length(p) for p in range(n)], dtype=np.uint64)
    padded = (lens + np.uint64(255)) // np.uint64(256) * np.uint64(256)
    offs = np.concatenate([[0], np.cumsum(padded)[:-1]]).astype(np.uint64)
    total = int(offs[-1] + lens[-1]) + 256
    assert 130 << 30 < total < 150 << 30  # ~138 GiB, BASELINE configs[2]
    data = torch.empty(total, dtype=torch.uint8, device="cuda")
    try:
        s3.generate_parts(data, offs, lens, np.arange(n), SEED)
        with s3.Plan(offs, lens) as plan:
            info = plan.info()
            # 512 groups: two per workgroup, except the solo ones the makespan model adds
            assert info["kernel"] == "skew" and info["groups"] == 512 and info["solo"] > 0, info
            assert info["grid"] == info["solo"] + (512 - info["solo"] + 1) // 2, info
            out = torch.empty((n, 8), dtype=torch.int32, device="cuda")
            plan.launch(data, out)
            plan.status()
        got = out.cpu().numpy().view(np.uint32)
        txt = s3.digests_to_text(got)
        fx = golden["c3_parts"]
        assert {e["p"] for e in fx} >= {int(np.argmax(lens)), int(np.argmin(lens))}
        for e in fx:
            assert int(lens[e["p"]]) == e["L"] and txt[e["p"]] == e["digest"], e["p"]
        # the SHA-256 + MD5 pass over the same parts: the mixed grid (skew groups with self-fed
        # MD5 waves for the longest parts, skewp groups for the rest), every part checked
        assert 0 < info["dual_solo"] < 512, info
        sha, m5 = s3.sha256_md5_batch_device(data, offs, lens)
        torch.cuda.synchronize()
        want_sha, want_md5 = _oracle_whole(torch, oracle, data, offs, lens, md5=True)
        bad = np.flatnonzero((got != want_sha).any(axis=1))
        assert bad.size == 0, f"{bad.size} of {n} C3 digests differ from the oracle, e.g. {bad[:8]}"
        assert np.array_equal(sha.cpu().numpy().view(np.uint32), want_sha)
        m5h = m5.cpu().numpy().view(np.uint32)
        bad = np.flatnonzero((m5h != want_md5).any(axis=1))
        assert bad.size == 0, f"{bad.size} of {n} C3 MD5 digests differ, e.g. {bad[:8]}"
        mfx = golden["md5"]["c3_parts"]
        assert [s3.digests_to_text(m5h[e["p"]:e["p"] + 1], 4)[0] for e in mfx] == [e["digest"] for e in mfx]
        del sha, m5
    finally:
        del data
        _release(torch)


def test_c4_rank0_shard(torch_cuda, oracle, golden):
    torch = torch_cuda
    world, rank, per = 8, 0, 8192
    ids = np.arange(rank, per * world, world, dtype=np.uint64)       # global parts p % 8 == 0
    from s3client_amd.shard import shard_ids
    assert np.array_equal(ids, shard_ids(per * world, rank, world))
    L = 8 * MIB
    lens = np.full(per, L, dtype=np.uint64)
    offs = np.arange(per, dtype=np.uint64) * np.uint64(L)
    data = torch.empty(per * L, dtype=torch.uint8, device="cuda")     # 64 GiB
    try:
        s3.generate_parts(data, offs, lens, ids, SEED)
        with s3.Plan(offs, lens) as plan:  # AUTO: shared-SIMD producers, one workgroup per CU
            assert plan.info()["kernel"] == shared_range_kernel()
            assert plan.info()["grid"] == per // 32
            out = torch.empty((per, 8), dtype=torch.int32, device="cuda")
            plan.launch(data, out)
            torch.cuda.synchronize()
        with s3.Plan(offs, lens, kernel="skewp") as plan:  # the lane-pair kernel, same parts
            out2 = torch.empty((per, 8), dtype=torch.int32, device="cuda")
            plan.launch(data, out2)
            torch.cuda.synchronize()
        assert torch.equal(out, out2)
        got = out.cpu().numpy().view(np.uint32)
        txt = s3.digests_to_text(got)
        fx = [e for e in golden["c2_parts"] + golden["c4_parts"] if e["p"] % world == rank]
        assert len(fx) >= 7
        for e in fx:
            assert txt[e["p"] // world] == e["digest"], e["p"]
        want, _ = _oracle_whole(torch, oracle, data, offs, lens)
        bad = np.flatnonzero((got != want).any(axis=1))
        assert bad.size == 0, f"{bad.size} of {per} C4-shard digests differ, e.g. slots {bad[:8]}"
        # download verification at this size: the shard against its own
        # digests, then with one byte flipped in one part -- exactly that part mismatches
        n_bad, mask = s3.verify_batch_device(data, offs, lens, out)
        assert n_bad == 0 and not bool(mask.any())
        k = 5555
        pos = int(offs[k]) + L // 2 + 3
        data[pos] ^= 0x40
        n_bad, mask = s3.verify_batch_device(data, offs, lens, out)
        assert n_bad == 1 and np.flatnonzero(mask.cpu().numpy()).tolist() == [k]
    finally:
        del data
        _release(torch)


@pytest.mark.parametrize("cfg,world,rank", [("c4", 8, 7), ("c2", 4, 3), ("c4", 2, 1), ("c2", 8, 6)])
def test_other_rank_shards(torch_cuda, oracle, golden, cfg, world, rank):
    """The shard a rank other than 0 hashes in a multi-GPU run (bench.py, one process per GPU,
    global part p on rank p % N): BASELINE configs[3]'s rank 7 of 8, the C2 weak-scaling job's
    rank 3 of 4, and two more -- run here on the one GPU, checked against that rank's own
    lib/hash fixtures (gen_golden.py 4c: four slots per rank, plus any other fixture whose id
    falls in the shard), the oracle on 64 random parts and hashlib on every part."""
    torch = torch_cuda
    from s3client_amd.shard import shard_ids
    per = 8192 if cfg == "c4" else 1024
    ids = shard_ids(per * world, rank, world)
    L = 8 * MIB
    lens = np.full(per, L, dtype=np.uint64)
    offs = np.arange(per, dtype=np.uint64) * np.uint64(L)
    data = torch.empty(per * L, dtype=torch.uint8, device="cuda")
    try:
        s3.generate_parts(data, offs, lens, ids, SEED)
        with s3.Plan(offs, lens) as plan:
            assert plan.info()["kernel"] == (shared_range_kernel() if cfg == "c4" else "skew")
            out = torch.empty((per, 8), dtype=torch.int32, device="cuda")
            plan.launch(data, out)
            plan.status()  # device error word clear
        got = out.cpu().numpy().view(np.uint32)
        txt = s3.digests_to_text(got)
        own = [e for e in golden["shard_parts"]
               if e["cfg"] == cfg and e["N"] == world and e["rank"] == rank]
        assert len(own) == 4
        for e in own:
            assert int(ids[e["slot"]]) == e["p"] and txt[e["slot"]] == e["digest"], e
        slot_of = {int(p): k for k, p in enumerate(ids)}
        extra = [e for e in golden["c2_parts"] + golden["c4_parts"] + golden["shard_parts"]
                 if e["p"] in slot_of]
        for e in extra:
            assert txt[slot_of[e["p"]]] == e["digest"], e["p"]
        rng = np.random.default_rng(1000 * world + rank)
        slots = np.sort(rng.choice(per, 64, replace=False))
        assert np.array_equal(got[slots], _oracle_sample(torch, oracle, data, offs, lens, slots))
        bad = np.flatnonzero((got != _hashlib_whole(torch, data, offs, lens)).any(axis=1))
        assert bad.size == 0, f"{bad.size} of {per} digests differ, e.g. slots {bad[:8]}"
    finally:
        del data
        _release(torch)


@pytest.mark.parametrize("cfg", ["c4", "c2"])
def test_every_rank_of_eight_on_one_gpu(torch_cuda, oracle, golden, cfg):
    """BASELINE configs[3] whole: all 65,536 x 8 MiB parts (512 GiB) hashed shard by shard on
    the one GPU, each shard exactly as rank r of an 8-GPU run holds it (global part p on rank
    p % 8, slot p // 8), and the same for the C2 weak-scaling job at N = 8 (8,192 parts).  Every
    shard checked against its own lib/hash fixtures, the oracle on 16 random parts, and EVERY
    part against hashlib (all 65,536 digests of config 4); the multi-GPU run itself adds only
    concurrency on separate devices (no data-path exchange)."""
    torch = torch_cuda
    from s3client_amd.shard import shard_ids
    world, per, L = 8, (8192 if cfg == "c4" else 1024), 8 * MIB
    lens = np.full(per, L, dtype=np.uint64)
    offs = np.arange(per, dtype=np.uint64) * np.uint64(L)
    fx = {e["p"]: e["digest"] for e in golden["c2_parts"] + golden["c4_parts"] + golden["shard_parts"]}
    data = torch.empty(per * L, dtype=torch.uint8, device="cuda")
    out = torch.empty((per, 8), dtype=torch.int32, device="cuda")
    checked = 0
    try:
        with s3.Plan(offs, lens) as plan:
            for rank in range(world):
                ids = shard_ids(per * world, rank, world)
                s3.generate_parts(data, offs, lens, ids, SEED)
                plan.launch(data, out)
                plan.status()
                txt = s3.digests_to_text(out.cpu().numpy().view(np.uint32))
                mine = [k for k, p in enumerate(ids) if int(p) in fx]
                assert len(mine) >= 4, rank
                for k in mine:
                    assert txt[k] == fx[int(ids[k])], (rank, int(ids[k]))
                checked += len(mine)
                rng = np.random.default_rng(700 + rank)
                slots = np.sort(rng.choice(per, 16, replace=False))
                allgot = out.cpu().numpy().view(np.uint32)
                assert np.array_equal(allgot[slots], _oracle_sample(torch, oracle, data, offs, lens, slots)), rank
                bad = np.flatnonzero((allgot != _hashlib_whole(torch, data, offs, lens)).any(axis=1))
                assert bad.size == 0, f"rank {rank}: {bad.size} of {per} digests differ, e.g. {bad[:8]}"
        assert checked >= 4 * world
    finally:
        del data, out
        _release(torch)


def _ragged_top(rng, n, top, top_len, rest_len):
    lens = rng.integers(*rest_len, n)
    lens[:top] = rng.integers(*top_len, top)
    rng.shuffle(lens)
    offs = np.concatenate([[0], np.cumsum(lens + 3)[:-1]]).astype(np.uint64)  # misaligned
    return lens.astype(np.uint64), offs


def test_two_group_solo_grid(torch_cuda, oracle):
    """2,049-4,096 parts whose longest few set the time: the plan gives their groups solo
    workgroups, an equal-length batch gets none; one launch and resumable
    ranges (the host path's slices) both bit-exact vs the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(505)
    for n, top, top_len, rest_len, solo in ((4000, 150, (200_000, 300_000), (0, 40_000), True),
                                            (2600, 40, (110_000, 112_000), (1, 5_000), True),
                                            (4096, 0, (0, 1), (8192, 8193), False)):
        lens, offs = _ragged_top(rng, n, top, top_len, rest_len)
        host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
        data = torch.from_numpy(host).cuda()
        want = oracle.batch(host, offs, lens, threads=16)
        with s3.Plan(offs, lens) as plan:
            info = plan.info()
            groups = (n + 7) // 8
            assert info["kernel"] == "skew" and info["groups"] == groups, info
            assert (info["solo"] > 0) == solo, info
            assert info["grid"] == info["solo"] + (groups - info["solo"] + 1) // 2, info
            one = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
            plan.launch(data, one)
            many = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
            step = 1231
            for b0 in range(0, info["max_blocks"], step):
                plan.launch_range(data.data_ptr(), many, b0, b0 + step, 0)
            torch.cuda.synchronize()
        assert np.array_equal(one.cpu().numpy().view(np.uint32), want), n
        assert torch.equal(one, many), n
        del data
        _release(torch)


def test_64bit_lengths_and_offsets(torch_cuda):
    """Sizes past 32 bits: a part of 512 MiB + 7 B (its bit length, 2^32 + 56, has a non-zero
    high word in the padding, alloc_padded utility.cpp:42-56) and small parts placed beyond
    the 4 GiB byte offset of the device buffer, hashed by resumable launches of ~2 s each over
    block ranges (sha256_stream semantics).  Bit-exact vs hashlib."""
    import hashlib
    torch = torch_cuda
    big = 512 * MIB + 7
    lens = np.array([big, 0, 55, 64, 1000, 8 * MIB + 1], dtype=np.uint64)
    offs = np.array([0, (4 << 30) + 3, (4 << 30) + 256, (4 << 30) + 4096 + 1, (4 << 30) + 9000,
                     (4 << 30) + 16 * MIB], dtype=np.uint64)
    data = torch.empty(int(offs[-1] + lens[-1]) + 256, dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(61)
    for o, L in zip(offs, lens):
        if L:
            data[int(o):int(o) + int(L)] = torch.randint(0, 256, (int(L),), dtype=torch.uint8,
                                                         device="cuda", generator=g)
    want = [hashlib.sha256(data[int(o):int(o) + int(L)].cpu().numpy().tobytes()).hexdigest()
            for o, L in zip(offs, lens)]
    plan = s3.Plan(offs, lens)
    info = plan.info()
    assert info["max_blocks"] == (big + 9 + 63) // 64
    out = torch.zeros((len(lens), 8), dtype=torch.int32, device="cuda")
    step = 2 << 20  # blocks per launch: ~2 s of one chain
    for b in range(0, info["max_blocks"], step):
        plan.launch_range(data.data_ptr(), out, b, min(b + step, info["max_blocks"]), 0)
        torch.cuda.synchronize()
    assert s3.digests_to_text(out.cpu().numpy().view(np.uint32)) == want
    plan.close()
    del data, out
    _release(torch)
