"""The oracle (oracle/sha256_oracle.c) pinned against the reference's golden vectors.

tests/golden/sha256_golden.json was produced by tests/golden/gen_golden.py from the REAL
lib/hash compiled from /root/reference (and cross-checked there with hashlib)."""
import hashlib
import os
import hmac as pyhmac

import numpy as np
import pytest


def test_reference_kats(oracle, golden):
    # lib/hash/sha256.cpp:248-249, 284-285, 331-332 (+ empty, "abc")
    for k in golden["kat"]:
        assert oracle.hex(k["ascii"].encode()) == k["digest"], k["name"]


def test_kat_literals_from_reference_source(oracle):
    assert oracle.hex(b"12345678" * 6) == \
        "dd7f20ca4910f937c3e560427de36fea7c37eed94899b3a9bf286905860d17ae"
    assert oracle.hex(b"12345678" * 14 + b"1234567") == \
        "0c65765f1b9fff74bb831fa24c63d9ab0513c881fc7b4919b43f72f5487a24fd"
    assert oracle.hex(b"12345678" * 15) == \
        "979e3016a670a5b1308dba2d715f75201eebcef0adc4a1ac99877fad91ce3ff6"


def test_length_edges(oracle, golden):
    big = oracle.generate(7, max(e["L"] for e in golden["edge"]))
    for e in golden["edge"]:
        assert oracle.hex(big[:e["L"]]) == e["digest"], e["L"]


def test_generator_matches_c2_fixtures(oracle, golden):
    for e in golden["c2_parts"][:3]:
        assert oracle.hex(oracle.generate(e["p"], e["L"])) == e["digest"], e["p"]


def test_shard_fixtures(oracle, golden):
    """Every rank's shard fixtures at N = 2, 4, 8 (gen_golden.py 4c): p = slot * N + rank, four
    slots per rank, both the C2 weak-scaling job and C4; the oracle agrees on all of them."""
    from s3client_amd.shard import shard_ids
    sh = golden["shard_parts"]
    for cfg, per in (("c2", 1024), ("c4", 8192)):
        for N in (2, 4, 8):
            for r in range(N):
                mine = [e for e in sh if e["cfg"] == cfg and e["N"] == N and e["rank"] == r]
                assert len(mine) == 4, (cfg, N, r)
                ids = shard_ids(per * N, r, N)
                for e in mine:
                    assert int(ids[e["slot"]]) == e["p"] and e["p"] % N == r
    distinct = {e["p"]: e["digest"] for e in sh}
    blob = np.zeros((len(distinct), 8 << 20), dtype=np.uint8)
    for k, p in enumerate(distinct):
        blob[k] = np.frombuffer(oracle.generate(p, 8 << 20), dtype=np.uint8)
    got = oracle.batch(blob.reshape(-1), np.arange(len(distinct)) * (8 << 20),
                       np.full(len(distinct), 8 << 20))
    for k, (p, want) in enumerate(distinct.items()):
        assert got[k].tobytes().hex() == want, p


def test_c3_lengths(oracle, golden):
    assert [oracle.c3_length(p) for p in range(64)] == golden["c3_lengths"]
    assert golden["c3_lengths"][:4] == [52996377, 9123323, 20283550, 58275873]


def test_transfer_parts(oracle, golden):
    t = golden["transfer"]
    data = (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8).tobytes()
    for p in t["parts"]:
        assert oracle.hex(data[p["offset"]:p["offset"] + p["size"]]) == p["digest"]


def test_hmac(oracle, golden):
    for h in golden["hmac"]:
        assert oracle.hmac(bytes.fromhex(h["msg"]), bytes.fromhex(h["key"])).hex() == h["mac"]


def test_stream_state(oracle, golden):
    big = oracle.generate(7, 1000)
    iv = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
          0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
    for s in golden["stream"]:
        assert list(oracle.stream(iv, big[:s["L"]])) == s["state"], s["L"]


def test_batch_threads(oracle):
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 5000, 40)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    base = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    got = oracle.batch(base, offs, lens, threads=4)
    for i in range(40):
        want = hashlib.sha256(base[offs[i]:offs[i] + lens[i]].tobytes()).digest()
        assert got[i].tobytes() == want


def test_md5_oracle_golden(oracle, golden):
    import hashlib
    md = golden["md5"]
    big = oracle.generate(7, max(e["L"] for e in md["edge"]))
    for e in md["edge"]:
        assert oracle.md5(big[:e["L"]]).tobytes().hex() == e["digest"], e["L"]
    assert oracle.md5(b"").tobytes().hex() == hashlib.md5(b"").hexdigest()
    iv = [0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476]
    for s in md["stream"]:
        assert list(oracle.md5_stream(iv, big[:s["L"]])) == s["state"], s["L"]
    for e in md["c2_parts"][:1]:
        assert oracle.md5(oracle.generate(e["p"], e["L"])).tobytes().hex() == e["digest"]
    # C3 fixture parts (the shortest and part 0; the rest are checked on the GPU by bench.py)
    c3 = sorted(md["c3_parts"], key=lambda e: e["L"])
    for e in (c3[0], next(x for x in md["c3_parts"] if x["p"] == 0)):
        assert oracle.md5(oracle.generate(e["p"], e["L"])).tobytes().hex() == e["digest"], e["p"]


def test_cpu_baseline_restatement_matches_goldens(oracle, golden):
    """oracle/cpu_baseline.c (the lib/hash-cost-structure baseline bench.py times) is bit-exact
    on the reference KATs, every golden edge length (4 KiB scratch vs calloc'd copy) and a
    threaded batch of C2 parts."""
    import ctypes
    import subprocess
    import numpy as np
    from tests.oracle_lib import ROOT, u64p
    so = os.path.join(ROOT, "oracle", "libcpubase.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    L = ctypes.CDLL(so)
    L.base_sha256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    L.base_sha256_batch.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_int]

    def h(b: bytes) -> str:
        out = np.zeros(8, np.uint32)
        L.base_sha256(b, len(b), out.ctypes.data)
        return out.tobytes().hex()

    for k in golden["kat"]:
        assert h(k["ascii"].encode()) == k["digest"], k["name"]
    big = oracle.generate(7, max(e["L"] for e in golden["edge"]))
    for e in golden["edge"]:
        assert h(big[:e["L"]]) == e["digest"], e["L"]
    ps = [e for e in golden["c2_parts"]][:6]
    buf = np.concatenate([np.frombuffer(oracle.generate(e["p"], e["L"]), np.uint8) for e in ps])
    offs = np.arange(len(ps), dtype=np.uint64) * np.uint64(8 << 20)
    lens = np.full(len(ps), 8 << 20, dtype=np.uint64)
    out = np.zeros((len(ps), 8), np.uint32)
    assert L.base_sha256_batch(buf.ctypes.data, offs.ctypes.data_as(u64p), lens.ctypes.data_as(u64p),
                               len(ps), out.ctypes.data, 4) == 0
    assert [r.tobytes().hex() for r in out] == [e["digest"] for e in ps]
