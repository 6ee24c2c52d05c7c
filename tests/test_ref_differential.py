"""Differential fuzz against the REAL reference lib/hash (oracle/_ref/libref_hash.so, built from
/root/reference by oracle/Makefile).  Runs only where that library exists -- the build
container: oracle/_ref is git-ignored AND listed in .gpurunignore, so the reference's compiled
code never travels to the GPU box (and the test skips there).  Compares reference, oracle and
the product CPU drop-in on random lengths 0..64 KiB, block-boundary lengths and a few large
sizes."""
import ctypes
import hashlib
import os

import numpy as np
import pytest

import s3client_amd as s3
from tests.oracle_lib import REF_SO

pytestmark = pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built")


@pytest.fixture(scope="module")
def ref():
    L = ctypes.CDLL(REF_SO)
    L.ref_sha256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    L.ref_hmac256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                              ctypes.c_void_p]
    L.ref_sha256_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    return L


def _ref_digest(ref, b: bytes) -> np.ndarray:
    out = np.zeros(8, dtype=np.uint32)
    ref.ref_sha256(ctypes.create_string_buffer(b, len(b) or 1), len(b), out.ctypes.data)
    return out


def test_random_lengths(ref, oracle):
    rng = np.random.default_rng(99)
    lengths = list(rng.integers(0, 65536, 300)) + list(range(0, 200)) + [(1 << 20) + 7, 3 << 22]
    for L in lengths:
        b = rng.integers(0, 256, int(L), dtype=np.uint8).tobytes()
        want = _ref_digest(ref, b)
        assert np.array_equal(s3.sha256(b), want), L
        assert np.array_equal(oracle.sha256(b), want), L
        assert want.tobytes() == hashlib.sha256(b).digest()


def test_hmac_random_keys(ref, oracle):
    rng = np.random.default_rng(5)
    for _ in range(200):
        kl, ml = int(rng.integers(0, 65)), int(rng.integers(0, 300))
        k = rng.integers(0, 256, kl, dtype=np.uint8).tobytes()
        m = rng.integers(0, 256, ml, dtype=np.uint8).tobytes()
        out = ctypes.create_string_buffer(32)
        ref.ref_hmac256(ctypes.create_string_buffer(m, ml or 1), ml,
                        ctypes.create_string_buffer(k, kl or 1), kl, out)
        assert s3.hmac256(m, k) == out.raw == oracle.hmac(m, k), (kl, ml)


def test_stream_random(ref, oracle):
    rng = np.random.default_rng(6)
    iv = np.array([0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19], dtype=np.uint32)
    for L in list(rng.integers(0, 5000, 50)) + [0, 63, 64, 65]:
        b = rng.integers(0, 256, int(L), dtype=np.uint8).tobytes()
        st = iv.copy()
        ref.ref_sha256_stream(st.ctypes.data, ctypes.create_string_buffer(b, len(b) or 1), len(b))
        assert np.array_equal(oracle.stream(iv, b), st), L
