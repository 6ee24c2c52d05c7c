#!/usr/bin/env python3
"""Generate tests/golden/*.json from the REAL reference lib/hash (oracle/_ref/libref_hash.so).

Run in the build container (where /root/reference exists) after `make -C oracle`:

    python tests/golden/gen_golden.py

Every digest is computed by the compiled reference (`sha256::sha256`, `hmac256`) AND
independently by Python's hashlib/hmac; the script aborts if they ever disagree.  The JSON
holds data only (inputs are described by generator parameters, expected outputs as hex).
"""
import ctypes
import hashlib
import hmac
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SEED = 20241008


def load_ref():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_hash.so"))
    lib.ref_sha256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    lib.ref_hmac256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                ctypes.c_uint64, ctypes.c_void_p]
    lib.ref_sha256_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    lib.ref_md5_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    lib.ref_md5_file.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    return lib


def ref_md5(ref, buf: bytes) -> str:
    """MD5 via the reference's md5_file (md5.cpp:132-180; the only padded MD5 entry point)."""
    import tempfile
    with tempfile.NamedTemporaryFile(delete=False) as f:
        f.write(buf)
        path = f.name
    out = (ctypes.c_uint32 * 4)()
    ref.ref_md5_file(path.encode(), out)
    os.unlink(path)
    got = bytes(out).hex()
    assert got == hashlib.md5(buf).hexdigest(), (len(buf), got)
    return got


def load_oracle():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    lib.oracle_generate.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                    ctypes.c_void_p]
    lib.oracle_c3_length.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    lib.oracle_c3_length.restype = ctypes.c_uint64
    return lib


def ref_digest(ref, buf: bytes) -> str:
    out = (ctypes.c_uint32 * 8)()
    src = ctypes.create_string_buffer(buf, len(buf) or 1)
    ref.ref_sha256(src, len(buf), out)
    got = bytes(out).hex()  # words are bswap32(H_i): memory bytes == canonical digest
    want = hashlib.sha256(buf).hexdigest()
    assert got == want, (len(buf), got, want)
    return got


def gen(orc, p, L) -> bytes:
    out = ctypes.create_string_buffer(max(L, 1))
    orc.oracle_generate(SEED, p, L, out)
    return out.raw[:L]


def gen_py(p, L) -> bytes:
    """Independent numpy statement of generator G."""
    n = (L + 7) // 8
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    x0 = np.uint64((SEED ^ (p * 0xD1B54A32D192ED03)) & 0xFFFFFFFFFFFFFFFF)
    j = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x0 + j * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    del M
    return z.astype("<u8").tobytes()[:L]


def main():
    ref, orc = load_ref(), load_oracle()
    out = {"seed": SEED, "generator": "G(seed,p,L): SURVEY.md 8(d) splitmix64, little-endian"}

    # 1. the reference's own KATs (lib/hash/sha256.cpp:248-249, 284-285, 331-332) + empty
    kat = []
    for name, s in [("12345678x6", "12345678" * 6),
                    ("12345678x14+1234567", "12345678" * 14 + "1234567"),
                    ("12345678x15", "12345678" * 15),
                    ("empty", ""), ("abc", "abc")]:
        kat.append({"name": name, "ascii": s, "digest": ref_digest(ref, s.encode())})
    out["kat"] = kat

    # 2. length edges over G(SEED, 7, L)
    edges = [0, 1, 2, 3, 4, 5, 31, 32, 55, 56, 57, 58, 59, 60, 61, 62, 63, 64, 65, 100, 119, 120,
             121, 127, 128, 129, 183, 184, 191, 192, 1000, 4087, 4088, 4095, 4096, 4097, 5000,
             65535, 65536, 1 << 20, (1 << 20) + 13, 5242893, 8 << 20, (8 << 20) + 1]
    big = gen(orc, 7, max(edges))
    assert big[:100000] == gen_py(7, 100000)
    out["edge"] = [{"p": 7, "L": L, "digest": ref_digest(ref, big[:L])} for L in edges]

    # 3. 8 MiB parts of the C2 workload (part p = G(SEED, p, 8 MiB))
    L8 = 8 << 20
    ps = list(range(16)) + [511, 1022, 1023]
    out["c2_parts"] = [{"p": p, "L": L8, "digest": ref_digest(ref, gen(orc, p, L8))} for p in ps]

    # 4. C3 ragged lengths (first 64) + digests of whole C3 parts: p 0, 1, the longest and the
    #    shortest of the 4096, and four more spread over the batch (BASELINE configs[2])
    c3all = [int(orc.oracle_c3_length(SEED, p)) for p in range(4096)]
    out["c3_lengths"] = c3all[:64]
    c3ids = [0, 1, int(np.argmax(c3all)), int(np.argmin(c3all)), 777, 2048, 3000, 4095]
    out["c3_parts"] = [{"p": p, "L": c3all[p], "digest": ref_digest(ref, gen(orc, p, c3all[p]))}
                       for p in c3ids]

    # 4b. C4 (BASELINE configs[3]): 65536 x 8 MiB, part p on device p % 8.  Digests of parts of
    #     rank 0's shard (p = 8k) beyond the C2 fixtures, incl. its first, middle and last parts.
    out["c4_parts"] = [{"p": p, "L": 8 << 20, "digest": ref_digest(ref, gen(orc, p, 8 << 20))}
                       for p in (8, 16, 4096, 32768, 65520, 65528)]

    # 4c. Every rank's shard at N = 2, 4, 8 GPUs (global part p -> rank p % N, slot p // N;
    #     s3client_amd/shard.py): the C2 weak-scaling job (1,024 parts per GPU, ids < 1024 N)
    #     and C4 (8,192 per GPU, ids < 8192 N; N = 8 is BASELINE configs[3]).  Four slots per
    #     rank -- first, an odd one, the middle and the last -- so every rank of a multi-GPU run
    #     checks its own digests against lib/hash, not only the fixtures that happen to fall in
    #     its residue class.
    shards, seen = [], {}
    for cfg, per in (("c2", 1024), ("c4", 8192)):
        for N in (2, 4, 8):
            for r in range(N):
                for slot in (0, per // 4 + 1, per // 2, per - 1):
                    p = slot * N + r
                    if p not in seen:
                        seen[p] = ref_digest(ref, gen(orc, p, L8))
                    shards.append({"cfg": cfg, "N": N, "rank": r, "slot": slot, "p": p, "L": L8,
                                   "digest": seen[p]})
    out["shard_parts"] = shards

    # 5. test/parallel-file-transfer-test.cpp:50-59 data (i % 128, 38000007 B), parts sliced
    #    with lib/src/upload.cpp:98-107 geometry (3 jobs x 2 parts)
    size = 38000007
    data = (np.arange(size, dtype=np.uint64) % 128).astype(np.uint8).tobytes()
    parts = []
    jobs, ppj = 3, 2
    per_job = (size + jobs - 1) // jobs
    for job in range(jobs):
        off = job * per_job
        chunk = min(per_job, size - off)
        psz = (chunk + ppj - 1) // ppj
        for i in range(ppj):
            s = min(psz, chunk - i * psz)
            parts.append({"offset": off, "size": s, "digest": ref_digest(ref, data[off:off + s])})
            off += s
    out["transfer"] = {"size": size, "fill": "i%128", "jobs": jobs, "parts_per_job": ppj,
                       "parts": parts, "whole": ref_digest(ref, data)}

    # 6. test/api/multipart-upload{,-file}-test.cpp:47-54: 19000000 B iota (char wraps)
    size = 19000000
    data = (np.arange(size, dtype=np.uint64) % 256).astype(np.uint8).tobytes()
    mp = []
    for nchunks in (3, 2):
        cs = (size + nchunks - 1) // nchunks
        for i in range(nchunks):
            s = min(cs, size - cs * i)
            mp.append({"chunks": nchunks, "offset": i * cs, "size": s,
                       "digest": ref_digest(ref, data[i * cs:i * cs + s])})
    out["multipart"] = {"size": size, "fill": "i%256", "parts": mp}

    # 7. hmac256 (lib/hash/hmac256.cpp:60-95): key <= 64 across lengths; key > 64 only with
    #    message length == key length (the reference hashes `length` bytes of the key).
    hm = []
    rng = np.random.default_rng(SEED)
    for klen in (0, 1, 20, 32, 40, 44, 63, 64, 65, 100):
        for mlen in (0, 1, 8, 55, 56, 64, 100, 1000):
            if klen > 64 and mlen != klen:
                continue
            key = rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
            msg = rng.integers(0, 256, mlen, dtype=np.uint8).tobytes()
            o = (ctypes.c_uint8 * 32)()
            ref.ref_hmac256(ctypes.create_string_buffer(msg, mlen or 1), mlen,
                            ctypes.create_string_buffer(key, klen or 1), klen, o)
            want = hmac.new(key, msg, hashlib.sha256).hexdigest()
            assert bytes(o).hex() == want, (klen, mlen)
            hm.append({"key": key.hex(), "msg": msg.hex(), "mac": want})
    for klen in (100,):  # key > 64 and length == klen: the bug is invisible
        pass
    out["hmac"] = hm

    # 8. sha256_stream (lib/hash/sha256.cpp:84-144) state after whole blocks, tail ignored
    st = []
    for L in (0, 63, 64, 100, 128, 1000):
        h = (ctypes.c_uint32 * 8)(0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                  0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19)
        buf = big[:L]
        ref.ref_sha256_stream(h, ctypes.create_string_buffer(buf, L or 1), L)
        st.append({"p": 7, "L": L, "state": [int(x) for x in h]})
    out["stream"] = st

    # 9. MD5 (lib/hash/md5.cpp, SURVEY 8(f) "next"): md5_file digests (empty files make the
    #    reference exit, so L >= 1), md5_stream whole-block states, C2/transfer parts, ETag
    md = {"edge": [], "stream": [], "c2_parts": [], "c3_parts": [], "transfer": []}
    for L in [1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 128, 1000, 4096, 65536, (1 << 20) + 13,
              (16 << 20), (16 << 20) + 1]:
        md["edge"].append({"p": 7, "L": L, "digest": ref_md5(ref, big[:L] if L <= len(big)
                                                             else gen(orc, 7, L))})
    for L in (0, 64, 128, 640, 4096):
        h = (ctypes.c_uint32 * 4)(0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476)
        ref.ref_md5_stream(h, ctypes.create_string_buffer(big[:L], L or 1), L)
        md["stream"].append({"p": 7, "L": L, "state": [int(x) for x in h]})
    for p in (0, 1, 1023):
        md["c2_parts"].append({"p": p, "L": L8, "digest": ref_md5(ref, gen(orc, p, L8))})
    # the C3 fixture parts (the dual SHA-256 + MD5 pass over BASELINE configs[2])
    for p in c3ids:
        md["c3_parts"].append({"p": p, "L": c3all[p], "digest": ref_md5(ref, gen(orc, p, c3all[p]))})
    size = 38000007
    tdata = (np.arange(size, dtype=np.uint64) % 128).astype(np.uint8).tobytes()
    for prt in out["transfer"]["parts"]:
        o, n_ = prt["offset"], prt["size"]
        md["transfer"].append({"offset": o, "size": n_, "digest": ref_md5(ref, tdata[o:o + n_])})
    # S3 multipart ETag: hex(MD5(concat(binary part MD5s))) + "-" + part count
    cat = b"".join(bytes.fromhex(x["digest"]) for x in md["transfer"])
    md["transfer_etag"] = hashlib.md5(cat).hexdigest() + "-%d" % len(md["transfer"])
    out["md5"] = md

    path = os.path.join(HERE, "sha256_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    sys.exit(main())
