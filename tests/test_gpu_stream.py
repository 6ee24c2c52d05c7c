"""GPU parity of the multi-object stream (s3h_stream_*).

A stream appends chunks to n messages and finishes them with the documented sha256_next
contract (lib/hash/sha256.h:73-89): the digest must equal the one-shot digest of the
concatenation of every chunk (oracle_sha256 / oracle_md5 over the joined bytes), bit-exact,
for every chunk schedule -- empty chunks, chunks that stay inside one block, chunks that
complete a carried block exactly, multi-block chunks at any alignment."""
import os

import numpy as np
import pytest

import s3client_amd as s3

pytestmark = pytest.mark.gpu
KERNELS = ["skew", "skewp", "skews", "quad", "pair", "pc", "lane"]


def _schedule(rng, n, rounds, maxlen):
    """Per-round chunk lengths with the carry edge cases mixed in."""
    special = np.array([0, 1, 3, 55, 56, 63, 64, 65, 127, 128, 129, 200])
    out = []
    for _ in range(rounds):
        lens = rng.integers(0, maxlen, n)
        pick = rng.random(n) < 0.5
        lens[pick] = rng.choice(special, int(pick.sum()))
        out.append(lens)
    return out


def _oracle_digest(oracle, algo, data: bytes):
    return oracle.sha256(data) if algo == "sha256" else oracle.md5(data)


def _check_stream(oracle, algo, kernel, n, rounds, maxlen, seed, finals=2):
    rng = np.random.default_rng(seed)
    with s3.Stream(n, algo=algo, kernel=kernel) as st:
        for f in range(finals):
            msgs = [bytearray() for _ in range(n)]
            for lens in _schedule(rng, n, rounds, maxlen):
                chunks = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
                st.update(chunks)
                for i, c in enumerate(chunks):
                    msgs[i] += c
            assert all(st.total(i) == len(msgs[i]) for i in range(n))
            got = st.final()
            want = np.stack([_oracle_digest(oracle, algo, bytes(m)) for m in msgs])
            bad = [i for i in range(n) if not np.array_equal(got[i], want[i])]
            assert not bad, (f, bad[:8], [len(msgs[i]) for i in bad[:8]])
            assert all(st.total(i) == 0 for i in range(n))  # final() restarts the messages


@pytest.mark.parametrize("kernel", KERNELS)
def test_stream_sha256_random_schedules(torch_cuda, oracle, kernel):
    _check_stream(oracle, "sha256", kernel, n=150, rounds=6, maxlen=3000, seed=11)


def test_stream_md5_random_schedules(torch_cuda, oracle):
    _check_stream(oracle, "md5", "auto", n=150, rounds=6, maxlen=3000, seed=12)


def test_stream_empty_messages(torch_cuda, oracle):
    """No update at all / only empty chunks: the digest of the empty message."""
    with s3.Stream(5) as st:
        got = st.final()
        st.update([b""] * 5)
        got2 = st.final()
    want = oracle.sha256(b"")
    assert all(np.array_equal(g, want) for g in got) and np.array_equal(got, got2)
    with s3.Stream(3, algo="md5") as st:
        assert all(np.array_equal(g, oracle.md5(b"")) for g in st.final())


def test_stream_device_chunks_unaligned(torch_cuda, oracle):
    """update_device: chunks at arbitrary offsets of a device tensor, final into HBM."""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    n, rounds = 64, 5
    msgs = [bytearray() for _ in range(n)]
    with s3.Stream(n) as st:
        for lens in _schedule(rng, n, rounds, 70000):
            gaps = rng.integers(0, 8, n)
            offs = np.cumsum(gaps + np.concatenate([[0], lens[:-1]]))
            host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 1, dtype=np.uint8)
            data = torch.from_numpy(host).cuda()
            st.update_device(data, offs, lens)
            torch.cuda.synchronize()
            for i in range(n):
                msgs[i] += host[offs[i]:offs[i] + lens[i]].tobytes()
        out = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
        st.final_device(out)
        torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    want = np.stack([oracle.sha256(bytes(m)) for m in msgs])
    assert np.array_equal(got, want)


def test_stream_large_objects_match_batch(torch_cuda, oracle, golden):
    """Eight 8 MiB C2 parts streamed in ragged chunks (1 B .. 3 MiB) hash to the golden
    one-shot digests of lib/hash (tests/golden c2_parts)."""
    parts = golden["c2_parts"][:8]
    bufs = [np.frombuffer(oracle.generate(p["p"], p["L"]), dtype=np.uint8) for p in parts]
    rng = np.random.default_rng(9)
    pos = [0] * len(bufs)
    with s3.Stream(len(bufs)) as st:
        while any(pos[i] < bufs[i].size for i in range(len(bufs))):
            chunks = []
            for i, b in enumerate(bufs):
                L = int(rng.choice([1, 63, 64, 4097, 1 << 20, 3 << 20]))
                chunks.append(b[pos[i]:pos[i] + L])
                pos[i] = min(pos[i] + L, b.size)
            st.update(chunks)
        got = s3.digests_to_text(st.final())
    assert got == [p["digest"] for p in parts]


def test_stream_many_messages_pc_lane_policy(torch_cuda, oracle):
    """n above the pair/pc thresholds: AUTO picks pc / lane plans for the stream too."""
    rng = np.random.default_rng(3)
    n = 70000
    lens1 = rng.integers(0, 150, n)
    lens2 = rng.integers(0, 150, n)
    base1 = rng.integers(0, 256, int(lens1.sum()), dtype=np.uint8)
    base2 = rng.integers(0, 256, int(lens2.sum()), dtype=np.uint8)
    o1 = np.concatenate([[0], np.cumsum(lens1)[:-1]])
    o2 = np.concatenate([[0], np.cumsum(lens2)[:-1]])
    with s3.Stream(n) as st:
        st.update([base1[o1[i]:o1[i] + lens1[i]] for i in range(n)])
        st.update([base2[o2[i]:o2[i] + lens2[i]] for i in range(n)])
        got = st.final()
    # every message: the two chunks concatenated, hashed by the oracle as one batch
    cat = np.concatenate([np.concatenate([base1[o1[i]:o1[i] + lens1[i]], base2[o2[i]:o2[i] + lens2[i]]])
                          for i in range(n)])
    lens = lens1 + lens2
    want = oracle.batch(cat, np.concatenate([[0], np.cumsum(lens)[:-1]]), lens, threads=16)
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, f"{bad.size} of {n} streamed digests differ, e.g. {bad[:8]}"


@pytest.mark.parametrize("n", [6000, 12000])
def test_stream_shared_simd_and_lane_pair_ranges(torch_cuda, oracle, n):
    """Message counts in AUTO's shared-SIMD (4,097 - 8,192: skews) and lane-pair (8,193 -
    28,672: skewp) ranges: ragged appends (incl. empty and < 64 B carries), two finals, every
    digest vs the oracle."""
    _check_stream(oracle, "sha256", "auto", n=n, rounds=3, maxlen=5000, seed=n, finals=2)


def test_stream_two_group_grid_ragged_updates(torch_cuda, oracle):
    """3,000 messages (AUTO = the two-group skew kernel): every update re-sorts the plans and
    re-plans the solo workgroups for that update's ragged chunk lengths (plan_refill)."""
    _check_stream(oracle, "sha256", "auto", n=3000, rounds=3, maxlen=20000, seed=13, finals=1)


def test_concurrent_stream_objects(torch_cuda, oracle):
    """Four threads each drive their own stream object (objects uploaded as their chunks
    arrive, one per upload job) at the same time: SHA-256 on three, MD5 on one; every digest
    vs the oracle over the concatenated chunks."""
    import threading
    errors = []

    def job(k):
        try:
            _check_stream(oracle, "md5" if k == 3 else "sha256", "auto", 40 + 7 * k, 6, 20000,
                          seed=70 + k, finals=2)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(f"{k}: {e!r}")

    th = [threading.Thread(target=job, args=(k,)) for k in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors


@pytest.mark.parametrize("algo", ["sha256", "md5"])
def test_stream_messages_past_2_32_bits(torch_cuda, oracle, algo):
    """Messages longer than 512 MiB (bit length > 2^32: the final block's 64-bit length field
    uses its high word; sha256.cpp:147-160 / md5.cpp:132-180 padding) streamed from HBM in
    ragged chunks of up to 64 MiB, with the carry crossing every chunk boundary: digests vs
    the oracle over the same bytes."""
    torch = torch_cuda
    rng = np.random.default_rng(2 ** 32)
    total = (512 << 20) + 4099  # past 2^32 bits, ragged last block
    host = rng.integers(0, 256, total + 64, dtype=np.uint8)
    data = torch.from_numpy(host).cuda()
    n = 2  # message 1 is message 0 shifted by 7 bytes
    starts = [0, 7]
    pos = 0
    with s3.Stream(n, algo=algo) as st:
        while pos < total:
            L = min(int(rng.integers(1, 64 << 20)), total - pos)
            st.update_device(data, [starts[0] + pos, starts[1] + pos], [L, L])
            pos += L
        torch.cuda.synchronize()
        assert st.total(0) == total and st.total(1) == total
        got = st.final()
    for i, s0 in enumerate(starts):
        m = host[s0:s0 + total].tobytes()
        want = oracle.sha256(m) if algo == "sha256" else oracle.md5(m)
        assert np.array_equal(got[i], want), (algo, i)


def test_stream_updates_on_alternating_streams(torch_cuda, oracle):
    """Back-to-back device updates issued on two different HIP streams in turn, with no host
    sync between them (the host prepares update k+1 while update k runs): every update is
    ordered after the previous one on the device, so the digests equal the oracle's over the
    concatenated chunks."""
    torch = torch_cuda
    rng = np.random.default_rng(91)
    n, rounds = 300, 12
    lens_r = _schedule(rng, n, rounds, 200000)
    total = [int(sum(l[i] for l in lens_r)) for i in range(n)]
    host = rng.integers(0, 256, sum(total) + 64, dtype=np.uint8)
    data = torch.from_numpy(host).cuda()
    starts = np.concatenate([[0], np.cumsum(total)[:-1]]).astype(np.int64)
    pos = np.zeros(n, dtype=np.int64)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    out = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
    with s3.Stream(n) as st:
        for k, lens in enumerate(lens_r):
            st.update_device(data, (starts + pos).astype(np.uint64), lens, streams[k % 2])
            pos += lens
        st.final_device(out, streams[0])
        torch.cuda.synchronize()
        st.status(streams[0])
    want = oracle.batch(host, starts, np.array(total), threads=16)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_stream_host_updates_from_buffer_parts(torch_cuda, oracle):
    """Host-form updates whose chunks are BufferParts ranges of one host buffer (pointers
    formed in numpy): digests equal the oracle's over the concatenated chunks."""
    rng = np.random.default_rng(77)
    n, rounds = 200, 4
    lens_r = _schedule(rng, n, rounds, 30000)
    msgs = [bytearray() for _ in range(n)]
    with s3.Stream(n) as st:
        for lens in lens_r:
            buf = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
            st.update(s3.BufferParts(buf, offs, lens))
            for i in range(n):
                msgs[i] += buf[offs[i]:offs[i] + lens[i]].tobytes()
        got = st.final()
    want = np.stack([oracle.sha256(bytes(m)) for m in msgs])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("chunk", [64 << 10, 1000, 4096 + 17])
@pytest.mark.parametrize("alternate", [False, True])
def test_stream_equal_chunks_reuse_device_slots(torch_cuda, oracle, chunk, alternate):
    """Equal-length device chunks appended at advancing offsets (the usual streamed upload):
    an update whose lengths equal the ones in the plan's device slots and whose offsets are
    those plus one constant launches on the same slots with the base moved by that constant
    (capi.hip stream_plan_base).  Chunk sizes that are a multiple of 64 B (the body plan is
    reused on every update after the first) and ones that are not (a carry at every
    boundary: the head plan's slots are reused), on one HIP stream and on two in turn, with
    two finals; messages start at unrelated byte offsets; every digest vs the oracle, and the
    slot-reuse counter shows the path was taken."""
    torch = torch_cuda
    rng = np.random.default_rng(chunk + alternate)
    n, rounds, finals = 96, 9, 2
    span = rounds * chunk
    starts = (np.arange(n, dtype=np.int64) * (span + 13) + rng.integers(0, 64, n)).astype(np.int64)
    host = rng.integers(0, 256, int(starts[-1]) + span + 64, dtype=np.uint8)
    data = torch.from_numpy(host).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    lens = np.full(n, chunk, dtype=np.uint64)
    want = oracle.batch(host, starts, np.full(n, span), threads=16)
    with s3.Stream(n) as st:
        for f in range(finals):
            for k in range(rounds):
                s = streams[k % 2] if alternate else streams[0]
                st.update_device(data, (starts + k * chunk).astype(np.uint64), lens, s)
            out = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
            st.final_device(out, streams[0])
            torch.cuda.synchronize()
            st.status(streams[0])
            got = out.cpu().numpy().view(np.uint32)
            bad = np.flatnonzero((got != want).any(axis=1))
            assert bad.size == 0, (f, bad[:8])
        stats = st.stats()
    # multiple of 64: body slots reused on every update after the first of each final round;
    # otherwise the heads (64 B at 64*i in the splice buffer) reuse theirs
    assert stats["slot_reuses"] >= (finals * (rounds - 1) if chunk % 64 == 0 else rounds - 2), stats


@pytest.mark.parametrize("pinned,equal,n", [(False, False, 64), (True, False, 64), (True, True, 64),
                                           (True, False, 100), (False, True, 100)])
def test_stream_host_updates_pipelined_and_buffer_reuse(torch_cuda, oracle, pinned, equal, n):
    """Host-form updates copy the chunks out and return while the hash still runs; the next
    update's copy overlaps it (two device staging sets).  Copy forms: pinned chunks of equal
    length at one stride -> one 2-D DMA; up to 64 other pinned chunks -> one DMA each; more, or
    pageable ones -> copy threads through two pinned 64 MiB pieces; updates above 256 MiB
    (100 x 4 MiB) are appended as sub-updates.  The caller overwrites its one chunk buffer right
    after every update returns -- as an uploader reusing its read buffer does -- and the
    digests must still be those of the bytes it passed.  Empty and ragged chunks, staging
    regrowth, and a final in between that restarts the messages."""
    torch = torch_cuda
    rng = np.random.default_rng(404 + 2 * pinned + equal + n)
    cap = 4 << 20
    buf = torch.empty(n * cap, dtype=torch.uint8, pin_memory=pinned)
    view = buf.numpy()
    offs = np.arange(n, dtype=np.uint64) * np.uint64(cap)
    with s3.Stream(n) as st:
        for f, rounds in enumerate((3, 5)):
            msgs = [bytearray() for _ in range(n)]
            for k in range(rounds):
                top = [4096, 300000, 3 << 20, 4 << 20, 1 << 20][k % 5]
                if equal:
                    lens = np.full(n, top - 7 * (k % 2))  # a 64-B multiple or not
                else:
                    lens = rng.integers(0, top + 1, n)
                    lens[rng.integers(0, n, 3)] = 0
                view[:] = rng.integers(0, 256, view.size, dtype=np.uint8)
                for i in range(n):
                    msgs[i] += view[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
                st.update(s3.BufferParts(buf, offs, lens))
                view[:] = 0xA5  # the caller reuses its buffer at once
            got = st.final()
            want = np.stack([oracle.sha256(bytes(m)) for m in msgs])
            bad = [i for i in range(n) if not np.array_equal(got[i], want[i])]
            assert not bad, (f, bad[:8])


_SUB_FAIL_CHILD = r"""
import sys, json
sys.path.insert(0, sys.argv[1])
import os

import numpy as np
import s3client_amd as s3
from tests.oracle_lib import Oracle
rng = np.random.default_rng(31)
big = [rng.integers(0, 256, 200 << 20, dtype=np.uint8) for _ in range(2)]  # 4 sub-updates each
small = [rng.integers(0, 256, 1000 + i, dtype=np.uint8) for i in range(2)]
out = {}
st = s3.Stream(2)
try:
    st.update(big)
    out["first"] = 0
except s3.S3HashError as e:
    out["first"], out["first_msg"] = e.code, str(e)
try:
    st.update(small)
    out["second"] = 0
    out["digests_ok"] = bool(np.array_equal(st.final(), np.stack([Oracle().sha256(s.tobytes()) for s in small])))
except s3.S3HashError as e:
    out["second"], out["second_msg"] = e.code, str(e)
print(json.dumps(out))
"""


@pytest.mark.parametrize("fail_sub", [0, 1])
def test_stream_update_fails_midway(torch_cuda, fail_sub):
    """Advisor r5: a large host update is appended as sub-updates; when sub-update k fails
    (S3H_TEST_STREAM_FAIL_SUB injects it before its copy), the call returns the error after the
    copy stream has drained.  k > 0: the earlier sub-updates were appended, so the object is
    failed -- the next call returns S3H_EINVAL instead of appending those pieces twice.  k = 0:
    nothing was appended or queued, the object stays usable and its digests are right."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _SUB_FAIL_CHILD, root], capture_output=True, text=True,
                       timeout=300, cwd=root, env={**os.environ, "S3H_TEST_STREAM_FAIL_SUB": str(fail_sub)})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["first"] == -4 and f"injected failure of sub-update {fail_sub}" in out["first_msg"], out
    if fail_sub == 0:
        assert out["second"] == 0 and out["digests_ok"], out
    else:
        assert out["second"] == -1 and "failed earlier" in out["second_msg"], out
