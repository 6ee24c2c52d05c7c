"""ctypes loader for oracle/liboracle.so -- TEST INFRASTRUCTURE (the checker only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_hash.so")
SEED = 20241008
u64p = ctypes.POINTER(ctypes.c_uint64)


def _ensure_built():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)


class Oracle:
    def __init__(self):
        _ensure_built()
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_sha256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_sha256_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_hmac256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_generate.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_void_p]
        L.oracle_c3_length.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_c3_length.restype = ctypes.c_uint64
        L.oracle_sha256_batch.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_int]
        L.oracle_md5.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_md5_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_md5_batch.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_int]
        self.L = L

    def md5(self, data: bytes) -> np.ndarray:
        out = np.zeros(4, dtype=np.uint32)
        b = bytes(data)
        self.L.oracle_md5(b, len(b), out.ctypes.data)
        return out

    def md5_stream(self, state, data: bytes) -> np.ndarray:
        st = np.array(state, dtype=np.uint32)
        b = bytes(data)
        self.L.oracle_md5_stream(st.ctypes.data, b, len(b))
        return st

    def md5_batch(self, base: np.ndarray, offsets, lengths, threads: int = 8) -> np.ndarray:
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lengths, dtype=np.uint64)
        out = np.zeros((offs.size, 4), dtype=np.uint32)
        self.L.oracle_md5_batch(base.ctypes.data, offs.ctypes.data_as(u64p),
                                lens.ctypes.data_as(u64p), offs.size, out.ctypes.data, threads)
        return out

    def sha256(self, data: bytes) -> np.ndarray:
        out = np.zeros(8, dtype=np.uint32)
        b = bytes(data)
        self.L.oracle_sha256(b, len(b), out.ctypes.data)
        return out

    def hex(self, data: bytes) -> str:
        return self.sha256(data).tobytes().hex()

    def stream(self, state, data: bytes) -> np.ndarray:
        st = np.array(state, dtype=np.uint32)
        b = bytes(data)
        self.L.oracle_sha256_stream(st.ctypes.data, b, len(b))
        return st

    def hmac(self, data: bytes, key: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.oracle_hmac256(bytes(data), len(data), bytes(key), len(key), out)
        return out.raw

    def generate(self, p: int, L: int, seed: int = SEED) -> bytes:
        out = ctypes.create_string_buffer(max(L, 1))
        self.L.oracle_generate(seed, p, L, out)
        return out.raw[:L]

    def c3_length(self, p: int, seed: int = SEED) -> int:
        return int(self.L.oracle_c3_length(seed, p))

    def batch(self, base: np.ndarray, offsets, lengths, threads: int = 8) -> np.ndarray:
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lengths, dtype=np.uint64)
        out = np.zeros((offs.size, 8), dtype=np.uint32)
        self.L.oracle_sha256_batch(base.ctypes.data, offs.ctypes.data_as(u64p),
                                   lens.ctypes.data_as(u64p), offs.size, out.ctypes.data, threads)
        return out
