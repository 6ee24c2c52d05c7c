"""Python view of the MI355X batched SHA-256 path (over the C-ABI, include/s3hash.h).

Mirrors lib/hash's interface (/root/reference/lib/hash/sha256.h):
  * ``sha256(data)``        -> 8 digest words, ``hash[i] = bswap32(H_i)`` (sha256.h:70, CPU)
  * ``hmac256(data, key)``  -> 32-byte MAC (hmac256.cpp:60-95, CPU)
  * ``hash_to_text(words)`` -> 64 lowercase hex chars (sha256.h:113-119)
and adds the batched GPU entry points that the parallel upload uses for per-part payload
hashes (lib/src/upload.cpp:89-110 -> S3Api::UploadFilePart(..., payloadHash)):
  * ``Plan`` / ``sha256_batch_device``  -- parts already resident in HBM (torch tensors)
  * ``sha256_batch_host``               -- parts in host memory, sharded over GPUs
  * ``sha256_md5_batch_{host,device}``  -- both digests (x-amz-content-sha256 + Content-MD5)
                                           from one pass over the parts

Device memory, streams and events come from PyTorch (plumbing only); all hashing is done by
the HIP kernels in s3client_amd/csrc.  Nothing here falls back to the CPU for a batch.
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, Sequence

import numpy as np

from . import _native
from ._native import check, lib

DIGEST_WORDS = 8


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def _p64(a: np.ndarray):
    return a.ctypes.data_as(_native.u64p)


def device_count() -> int:
    c = ctypes.c_int(0)
    rc = lib().s3h_device_count(ctypes.byref(c))
    return c.value if rc == 0 else 0


def device_pci_bus_id(device: int) -> str:
    """PCI address "dddd:bb:dd.f" of HIP device ``device`` (s3h_device_pci_bus_id)."""
    buf = ctypes.create_string_buffer(64)
    check(lib().s3h_device_pci_bus_id(device, buf, len(buf)))
    return buf.value.decode()


def nblocks(length: int) -> int:
    """64-byte compressions SHA-256 performs on a message of ``length`` bytes."""
    return (int(length) + 72) // 64


def _stream_handle(stream) -> int | None:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


class Plan:
    """Geometry of one batch of parts, uploaded once (s3h_plan_create)."""

    def __init__(self, offsets: Sequence[int], lengths: Sequence[int], device: int = 0,
                 kernel: str | int = "auto", algo: str = "sha256"):
        k = kernel if isinstance(kernel, int) else _native.KERNEL_IDS[kernel]
        self.algo = _native.ALGO_IDS[algo]
        self.words = _native.DIGEST_WORDS[self.algo]
        self.offsets, self.lengths = _u64(offsets), _u64(lengths)
        if self.offsets.shape != self.lengths.shape or self.offsets.ndim != 1:
            raise ValueError("offsets and lengths must be 1-D and of equal length")
        self.n = int(self.lengths.size)
        self.device = device
        h = ctypes.c_void_p()
        check(lib().s3h_plan_create_ex(device, self.algo, _p64(self.offsets), _p64(self.lengths),
                                       self.n, k, ctypes.byref(h)))
        self._h = h

    def info(self) -> dict:
        n, tb, mb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        k, g = ctypes.c_int(), ctypes.c_uint32()
        check(lib().s3h_plan_info(self._h, ctypes.byref(n), ctypes.byref(tb), ctypes.byref(mb),
                                  ctypes.byref(k), ctypes.byref(g)))
        groups, solo = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().s3h_plan_groups(self._h, ctypes.byref(groups), ctypes.byref(solo)))
        dual_solo, apart = ctypes.c_uint32(), ctypes.c_int()
        check(lib().s3h_plan_dual_layout(self._h, ctypes.byref(dual_solo), ctypes.byref(apart)))
        return {"n": n.value, "total_blocks": tb.value, "max_blocks": mb.value,
                "kernel": _native.KERNEL_NAMES[k.value], "grid": g.value,
                "groups": groups.value, "solo": solo.value, "dual_solo": dual_solo.value,
                "dual_apart": bool(apart.value)}

    def set_clock_probe(self, clocks=None) -> int:
        """Record per-consumer-wave clock counters on later launches (skew kernel only):
        ``clocks`` is a device int64 tensor of >= 4 x waves entries ({clk0, clk1, rt0, rt1}
        per wave, s_memtime / s_memrealtime); None switches the probe off.  Returns the
        number of consumer waves that record (0 if the plan's kernel does not)."""
        w = ctypes.c_uint32()
        ptr = ctypes.c_void_p(clocks.data_ptr() if clocks is not None else None)
        check(lib().s3h_plan_set_clock_probe(self._h, ptr, ctypes.byref(w)))
        if clocks is not None and clocks.numel() < 4 * w.value:
            lib().s3h_plan_set_clock_probe(self._h, None, None)
            raise ValueError(f"clock buffer needs {4 * w.value} int64 entries")
        return w.value

    def _check_buffers(self, data, digests):
        import torch
        if not (data.is_cuda and digests.is_cuda):
            raise ValueError("data and digests must be device tensors")
        if digests.numel() * digests.element_size() < 4 * self.words * self.n:
            raise ValueError(f"digests buffer too small (need n*{4 * self.words} bytes)")
        end = int((self.offsets + self.lengths).max()) if self.n else 0
        if data.numel() * data.element_size() < end:
            raise ValueError(f"data buffer ({data.numel() * data.element_size()} B) smaller "
                             f"than the plan's extent ({end} B)")
        del torch

    def launch(self, data, digests, stream=None) -> None:
        """Hash every part of ``data`` (device tensor) into ``digests`` (n*8 words)."""
        self._check_buffers(data, digests)
        check(lib().s3h_plan_launch(self._h, ctypes.c_void_p(data.data_ptr()),
                                    ctypes.c_void_p(digests.data_ptr()),
                                    ctypes.c_void_p(_stream_handle(stream))))

    def status(self, stream=None) -> None:
        """Wait for ``stream`` and raise S3HashError (S3H_EHIP, "synchronisation timeout") if a
        launch since the last check reported a fault through the plan's device error word --
        its digests are then invalid (s3h_plan_status).  Clears the word."""
        check(lib().s3h_plan_status(self._h, ctypes.c_void_p(_stream_handle(stream))))

    def launch_range(self, data_ptr: int, digests, blk_begin: int, blk_end: int,
                     blk_origin: int, stream=None) -> None:
        check(lib().s3h_plan_launch_range(self._h, ctypes.c_void_p(data_ptr),
                                          ctypes.c_void_p(digests.data_ptr()), blk_begin,
                                          blk_end, blk_origin,
                                          ctypes.c_void_p(_stream_handle(stream))))

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().s3h_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def sha256_batch_device(data, offsets, lengths, device: int | None = None, kernel="auto",
                        stream=None, algo: str = "sha256"):
    """Digest every part [offsets[i], offsets[i]+lengths[i]) of the device tensor ``data``.

    Returns an (n, 8) int32 device tensor holding the uint32 digest words (lib/hash layout);
    (n, 4) for algo="md5"."""
    import torch
    dev = data.device.index if device is None else device
    with Plan(offsets, lengths, device=dev, kernel=kernel, algo=algo) as plan:
        out = torch.empty((plan.n, plan.words), dtype=torch.int32, device=data.device)
        plan.launch(data, out, stream)
        plan.status(stream)  # waits for the launch; raises if it reported a fault
    return out


def md5_batch_device(data, offsets, lengths, device: int | None = None, stream=None):
    """Batched MD5 of device-resident parts: (n, 4) int32 device tensor (LE digest words)."""
    return sha256_batch_device(data, offsets, lengths, device, "auto", stream, algo="md5")


def _as_bytes(p) -> np.ndarray:
    if type(p) is np.ndarray and p.dtype == np.uint8 and p.ndim == 1 and p.flags.c_contiguous:
        return p
    if isinstance(p, (bytes, bytearray, memoryview)):
        return np.frombuffer(p, dtype=np.uint8)
    return np.ascontiguousarray(p, dtype=np.uint8).reshape(-1)


def _addr(a: np.ndarray) -> int:
    # c_char.from_buffer is ~3x cheaper than a.ctypes.data / __array_interface__ (which build
    # objects per part: ~2 ms of a 1,024-part call); it needs a writable, non-empty buffer
    if not a.size:
        return 0
    if a.flags.writeable:
        return ctypes.addressof(ctypes.c_char.from_buffer(a))
    return a.__array_interface__["data"][0]


class BufferParts:
    """Host parts given as (offset, length) ranges of ONE host buffer -- a numpy uint8 array or
    a CPU torch tensor (pinned or pageable) -- usable wherever the host entry points take a
    sequence of parts.  The part pointers are formed in numpy, with no Python object per part
    (a 1,024-part call marshals in ~0.02 ms instead of ~0.5 ms for a list of views)."""

    def __init__(self, buf, offsets, lengths):
        if hasattr(buf, "data_ptr"):  # torch tensor
            if buf.is_cuda:
                raise ValueError("BufferParts takes host memory (use the *_device calls for HBM)")
            if not buf.is_contiguous():
                raise ValueError("BufferParts needs a contiguous buffer")
            base, size = buf.data_ptr(), buf.numel() * buf.element_size()
        else:
            buf = _as_bytes(buf)
            base, size = (buf.ctypes.data if buf.size else 0), int(buf.size)
        self._keep = buf
        offs, lens = _u64(offsets), _u64(lengths)
        if offs.shape != lens.shape or offs.ndim != 1:
            raise ValueError("offsets and lengths must be 1-D and of equal length")
        sz = np.uint64(size)
        if bool(((lens > 0) & ((offs > sz) | (lens > sz - np.minimum(offs, sz)))).any()):
            raise ValueError("a part extends past the end of the buffer")
        self.lens = lens
        self.addrs = np.where(lens > 0, offs + np.uint64(base), np.uint64(0)).astype(np.uint64)
        self.ptrs = self.addrs.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p))

    def __len__(self) -> int:
        return int(self.lens.size)


def _host_parts(parts):
    if isinstance(parts, BufferParts):
        return parts, parts.ptrs, parts.lens
    arrs = [_as_bytes(p) for p in parts]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * n)(*[_addr(a) for a in arrs])
    return arrs, ptrs, np.fromiter((a.size for a in arrs), dtype=np.uint64, count=n)


def _host_batch(fn, words, parts, ndevices, slice_bytes):
    arrs, ptrs, lens = _host_parts(parts)
    n = len(arrs)
    out = np.zeros((n, words), dtype=np.uint32)
    check(fn(ptrs, _p64(lens), n, out.ctypes.data, ndevices, slice_bytes))
    return out


def sha256_md5_batch_host(parts: Sequence, ndevices: int = 0,
                          slice_bytes: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """SHA-256 (n, 8) and MD5 (n, 4) uint32 digests of host-resident parts, each part crossing
    PCIe once (s3h_sha256_md5_batch_host)."""
    arrs, ptrs, lens = _host_parts(parts)
    n = len(arrs)
    sha = np.zeros((n, 8), dtype=np.uint32)
    m5 = np.zeros((n, 4), dtype=np.uint32)
    check(lib().s3h_sha256_md5_batch_host(ptrs, _p64(lens), n, sha.ctypes.data, m5.ctypes.data,
                                          ndevices, slice_bytes))
    return sha, m5


def sha256_md5_batch_device(data, offsets, lengths, device: int | None = None, stream=None):
    """SHA-256 (n, 8) and MD5 (n, 4) int32 device tensors of device-resident parts
    (s3h_sha256_md5_batch_device): one grid running both chains while the batch fits one
    workgroup per CU, above that the two kernels one after the other on ``stream``."""
    import torch
    dev = data.device.index if device is None else device
    offs, lens = _u64(offsets), _u64(lengths)
    if offs.shape != lens.shape:
        raise ValueError("offsets and lengths differ in length")
    n = int(lens.size)
    if n and int((offs + lens).max()) > data.numel() * data.element_size():
        raise ValueError("a part extends past the end of the data tensor")
    sha = torch.empty((n, 8), dtype=torch.int32, device=data.device)
    m5 = torch.empty((n, 4), dtype=torch.int32, device=data.device)
    check(lib().s3h_sha256_md5_batch_device(dev, data.data_ptr(), _p64(offs), _p64(lens), n,
                                            sha.data_ptr(), m5.data_ptr(),
                                            _stream_handle(stream)))
    return sha, m5


def md5_batch_host(parts: Sequence, ndevices: int = 0, slice_bytes: int = 0) -> np.ndarray:
    """Batched MD5 of host-resident parts on the GPUs: (n, 4) uint32."""
    return _host_batch(lib().s3h_md5_batch_host, 4, parts, ndevices, slice_bytes)


def verify_batch_host(parts: Sequence, expected, algo: str = "sha256",
                      ndevices: int = 0) -> np.ndarray:
    """Download-side verification: bool mask of parts whose digest differs from ``expected``
    ((n, 8) uint32 SHA-256 or (n, 4) MD5 words, or a list of hex strings)."""
    a = _native.ALGO_IDS[algo]
    words = _native.DIGEST_WORDS[a]
    if len(expected) and isinstance(expected[0], str):
        expected = np.stack([np.frombuffer(bytes.fromhex(h), dtype=np.uint32) for h in expected])
    exp = np.ascontiguousarray(expected, dtype=np.uint32).reshape(-1, words)
    arrs, ptrs, lens = _host_parts(parts)
    n = len(arrs)
    if exp.shape[0] != n:
        raise ValueError("expected digest count differs from part count")
    mism = np.zeros(n, dtype=np.uint8)
    cnt = ctypes.c_uint64(0)
    check(lib().s3h_verify_batch_host(a, ptrs, _p64(lens), n, exp.ctypes.data, mism.ctypes.data,
                                      ctypes.byref(cnt), ndevices))
    assert cnt.value == int(mism.sum())
    return mism.astype(bool)


def verify_batch_routed(parts: Sequence, expected, algo: str = "sha256", ndevices: int = 0,
                        route: str = "auto") -> tuple[np.ndarray, str]:
    """verify_batch_host on a route (s3h_verify_batch_routed): "gpu", "cpu", "split" or "auto"
    as sha256_batch_routed / md5_batch_routed, for either algorithm.  Returns (bool mismatch
    mask, route taken)."""
    a = _native.ALGO_IDS[algo]
    words = _native.DIGEST_WORDS[a]
    if len(expected) and isinstance(expected[0], str):
        expected = np.stack([np.frombuffer(bytes.fromhex(h), dtype=np.uint32) for h in expected])
    exp = np.ascontiguousarray(expected, dtype=np.uint32).reshape(-1, words)
    arrs, ptrs, lens = _host_parts(parts)
    n = len(arrs)
    if exp.shape[0] != n:
        raise ValueError("expected digest count differs from part count")
    mism = np.zeros(n, dtype=np.uint8)
    cnt = ctypes.c_uint64(0)
    taken = ctypes.c_int(-1)
    check(lib().s3h_verify_batch_routed(a, ptrs, _p64(lens), n, exp.ctypes.data, mism.ctypes.data,
                                        ctypes.byref(cnt), ndevices, _native.ROUTE_IDS[route],
                                        ctypes.byref(taken)))
    assert cnt.value == int(mism.sum())
    return mism.astype(bool), _native.ROUTE_NAMES[taken.value]


def verify_batch_device(data, offsets, lengths, expected, algo: str = "sha256", stream=None):
    """Device-resident verification: returns (mismatch count, bool mask on the device)."""
    import torch
    a = _native.ALGO_IDS[algo]
    offs, lens = _u64(offsets), _u64(lengths)
    mism = torch.zeros(offs.size, dtype=torch.uint8, device=data.device)
    cnt = ctypes.c_uint64(0)
    check(lib().s3h_verify_batch_device(data.device.index, a, ctypes.c_void_p(data.data_ptr()),
                                        _p64(offs), _p64(lens), offs.size,
                                        ctypes.c_void_p(expected.data_ptr()),
                                        ctypes.c_void_p(mism.data_ptr()), ctypes.byref(cnt),
                                        ctypes.c_void_p(_stream_handle(stream))))
    return cnt.value, mism.bool()


def multipart_etag(part_md5s) -> str:
    """S3 multipart ETag: hex(MD5(concatenated binary part MD5s)) + "-" + part count
    (s3h_multipart_etag; the outer MD5, 16 B per part, runs on the lib/hash MD5 drop-in)."""
    w = np.ascontiguousarray(part_md5s, dtype=np.uint32).reshape(-1, 4)
    out = ctypes.create_string_buffer(56)
    check(lib().s3h_multipart_etag(w.ctypes.data, w.shape[0], out, len(out)))
    return out.value.decode()


class Stream:
    """n messages (objects) hashed incrementally on the GPU as chunks arrive
    (s3h_stream_*, include/s3hash.h): sha256_stream semantics per append and the documented
    sha256_next contract (lib/hash/sha256.h:73-89) at ``final()`` -- the digest of the
    concatenation of every chunk appended since the previous ``final()``.

    ``update(chunks)`` takes one chunk per message: host ``bytes``/numpy arrays or
    ``BufferParts`` (returns once the chunks are copied; the hash overlaps the next update and
    ``final()`` reports a device fault of any of them), or, with ``update_device``, a device
    tensor plus offsets/lengths (asynchronous)."""

    def __init__(self, n: int, device: int = 0, algo: str = "sha256", kernel: str | int = "auto"):
        k = kernel if isinstance(kernel, int) else _native.KERNEL_IDS[kernel]
        self.algo = _native.ALGO_IDS[algo]
        self.words = _native.DIGEST_WORDS[self.algo]
        self.n, self.device = int(n), device
        h = ctypes.c_void_p()
        check(lib().s3h_stream_create(device, self.algo, self.n, k, ctypes.byref(h)))
        self._h = h

    def update(self, chunks: Sequence) -> None:
        if len(chunks) != self.n:
            raise ValueError(f"need one chunk per message ({self.n})")
        arrs, ptrs, lens = _host_parts(chunks)
        check(lib().s3h_stream_update_host(self._h, ptrs, _p64(lens)))

    def update_device(self, data, offsets, lengths, stream=None) -> None:
        offs, lens = _u64(offsets), _u64(lengths)
        if offs.size != self.n or lens.size != self.n:
            raise ValueError(f"need one chunk per message ({self.n})")
        if lens.any() and int((offs + lens)[lens > 0].max()) > data.numel() * data.element_size():
            raise ValueError("chunk extends past the data tensor")
        check(lib().s3h_stream_update_device(self._h, ctypes.c_void_p(data.data_ptr()),
                                             _p64(offs), _p64(lens),
                                             ctypes.c_void_p(_stream_handle(stream))))

    def final(self) -> np.ndarray:
        """(n, words) uint32 digests; the object restarts with n empty messages."""
        out = np.zeros((self.n, self.words), dtype=np.uint32)
        check(lib().s3h_stream_final_host(self._h, out.ctypes.data))
        return out

    def final_device(self, digests, stream=None) -> None:
        if digests.numel() * digests.element_size() < 4 * self.words * self.n:
            raise ValueError("digests buffer too small")
        check(lib().s3h_stream_final_device(self._h, ctypes.c_void_p(digests.data_ptr()),
                                            ctypes.c_void_p(_stream_handle(stream))))

    def status(self, stream=None) -> None:
        """Wait for ``stream``; raise if an update/final launch reported a fault
        (s3h_stream_status).  The host forms check by themselves."""
        check(lib().s3h_stream_status(self._h, ctypes.c_void_p(_stream_handle(stream))))

    def stats(self) -> dict:
        """How updates found their plans' device slots (s3h_stream_stats): reused in place
        (equal chunks appended at a moved base) or re-sorted and uploaded."""
        r, f = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().s3h_stream_stats(self._h, ctypes.byref(r), ctypes.byref(f)))
        return {"slot_reuses": r.value, "slot_refills": f.value}

    def total(self, i: int) -> int:
        t = ctypes.c_uint64()
        check(lib().s3h_stream_total(self._h, i, ctypes.byref(t)))
        return t.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().s3h_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def sha256_batch_host(parts: Sequence, ndevices: int = 0, slice_bytes: int = 0) -> np.ndarray:
    """Digest host-resident parts (bytes / numpy uint8 arrays) on the GPUs: (n, 8) uint32."""
    return _host_batch(lib().s3h_sha256_batch_host, DIGEST_WORDS, parts, ndevices, slice_bytes)


def sha256_batch_host_on(parts: Sequence, devices: Sequence[int], slice_bytes: int = 0) -> np.ndarray:
    """sha256_batch_host over an explicit device list (shard k = parts i % len(devices) == k on
    devices[k]; repeats allowed): s3h_sha256_batch_host_on."""
    arrs, ptrs, lens = _host_parts(parts)
    n = len(arrs)
    out = np.zeros((n, DIGEST_WORDS), dtype=np.uint32)
    devs = (ctypes.c_int * len(devices))(*devices)
    check(lib().s3h_sha256_batch_host_on(ptrs, _p64(lens), n, out.ctypes.data, devs, len(devices),
                                         slice_bytes))
    return out


def sha256_file_parts(path: str, offsets, lengths, ndevices: int = 0,
                      slice_bytes: int = 0) -> np.ndarray:
    """Digests of byte ranges [offsets[i], offsets[i]+lengths[i]) of a file, read by host
    threads straight into the pinned staging ring (s3h_sha256_file_parts): the (file, offset,
    size) parts of S3Api::UploadFilePart.  (n, 8) uint32."""
    offs, lens = _u64(offsets), _u64(lengths)
    if offs.shape != lens.shape or offs.ndim != 1 or offs.size == 0:
        raise ValueError("offsets and lengths must be 1-D, equal length and non-empty")
    out = np.zeros((offs.size, DIGEST_WORDS), dtype=np.uint32)
    check(lib().s3h_sha256_file_parts(os.fsencode(path), _p64(offs), _p64(lens), offs.size,
                                      out.ctypes.data, ndevices, slice_bytes))
    return out


def sha256_md5_file_parts(path: str, offsets, lengths, ndevices: int = 0,
                          slice_bytes: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """SHA-256 (n, 8) and MD5 (n, 4) uint32 digests of file ranges, each slice read once
    (s3h_sha256_md5_file_parts): x-amz-content-sha256 and Content-MD5 of UploadFilePart parts."""
    offs, lens = _u64(offsets), _u64(lengths)
    if offs.shape != lens.shape or offs.ndim != 1 or offs.size == 0:
        raise ValueError("offsets and lengths must be 1-D, equal length and non-empty")
    sha = np.zeros((offs.size, DIGEST_WORDS), dtype=np.uint32)
    m5 = np.zeros((offs.size, 4), dtype=np.uint32)
    check(lib().s3h_sha256_md5_file_parts(os.fsencode(path), _p64(offs), _p64(lens), offs.size,
                                          sha.ctypes.data, m5.ctypes.data, ndevices, slice_bytes))
    return sha, m5


def route_model() -> dict:
    """The size-aware routing model's rates, measured once per process on this host and GPU
    (s3h_route_model): per-thread CPU drop-in rate, one GPU chain's rate, pinned H2D rate,
    fixed GPU call cost, CPU threads, devices.  Raises S3HashError without a GPU."""
    m = _native.RouteModel()
    check(lib().s3h_route_model(ctypes.byref(m)))
    return {f: getattr(m, f) for f, _ in m._fields_}


def route_estimate(lengths, model: dict, ndevices: int = 0, pinned: bool = True,
                   source: str | None = None) -> tuple[str, float, float]:
    """AUTO's choice for a batch of parts of ``lengths`` under ``model`` (any dict with
    route_model()'s fields; pure host arithmetic, s3h_route_estimate_ex): (route, gpu_s,
    cpu_s).  ``source``: "pinned", "pageable" or "file" (default: pinned or pageable by
    ``pinned``) -- pageable parts and file ranges feed the GPU at min(h2d, staged)."""
    m = _native.RouteModel(**model)
    lens = _u64(lengths)
    src = _native.SOURCE_IDS[source or ("pinned" if pinned else "pageable")]
    g, c = ctypes.c_double(), ctypes.c_double()
    r = lib().s3h_route_estimate_ex(ctypes.byref(m), _p64(lens), lens.size, ndevices, src,
                                    ctypes.byref(g), ctypes.byref(c))
    if r < 0:
        check(r)
    return _native.ROUTE_NAMES[r], g.value, c.value


def route_split_estimate(lengths, model: dict, ndevices: int = 0,
                         source: str = "pinned") -> tuple[int, int, float]:
    """The split route's plan under ``model`` (s3h_route_split_estimate, pure host arithmetic):
    (m, tg, split_s) -- the m longest parts on the CPU, the rest on the GPU with tg staging
    threads per device (0 for pinned parts), estimated split_s seconds."""
    m = _native.RouteModel(**model)
    lens = _u64(lengths)
    k, tg, t = ctypes.c_uint64(), ctypes.c_int(), ctypes.c_double()
    check(lib().s3h_route_split_estimate(ctypes.byref(m), _p64(lens), lens.size, ndevices,
                                         _native.SOURCE_IDS[source], ctypes.byref(k), ctypes.byref(tg),
                                         ctypes.byref(t)))
    return k.value, tg.value, t.value


def sha256_batch_routed(parts: Sequence, ndevices: int = 0, route: str = "auto") -> tuple[np.ndarray, str]:
    """Host-resident parts hashed on the route given -- "gpu" (= sha256_batch_host), "cpu" (the
    lib/hash drop-in on host threads), "split" (the longest parts on the CPU, the rest on the
    GPU, at once) or "auto" (whichever the measured model says finishes first; needs a GPU) --
    s3h_sha256_batch_routed.  Returns ((n, 8) uint32, route taken)."""
    arrs, ptrs, lens = _host_parts(parts)
    out = np.zeros((len(arrs), DIGEST_WORDS), dtype=np.uint32)
    taken = ctypes.c_int(-1)
    check(lib().s3h_sha256_batch_routed(ptrs, _p64(lens), len(arrs), out.ctypes.data, ndevices,
                                        _native.ROUTE_IDS[route], ctypes.byref(taken)))
    return out, _native.ROUTE_NAMES[taken.value]


def sha256_file_parts_routed(path: str, offsets, lengths, ndevices: int = 0,
                             route: str = "auto") -> tuple[np.ndarray, str]:
    """File ranges on the route given (s3h_sha256_file_parts_routed): ((n, 8) uint32, taken)."""
    offs, lens = _u64(offsets), _u64(lengths)
    if offs.shape != lens.shape or offs.ndim != 1 or offs.size == 0:
        raise ValueError("offsets and lengths must be 1-D, equal length and non-empty")
    out = np.zeros((offs.size, DIGEST_WORDS), dtype=np.uint32)
    taken = ctypes.c_int(-1)
    check(lib().s3h_sha256_file_parts_routed(os.fsencode(path), _p64(offs), _p64(lens), offs.size,
                                             out.ctypes.data, ndevices, _native.ROUTE_IDS[route],
                                             ctypes.byref(taken)))
    return out, _native.ROUTE_NAMES[taken.value]


def md5_batch_routed(parts: Sequence, ndevices: int = 0, route: str = "auto") -> tuple[np.ndarray, str]:
    """Content-MD5 of host parts on a route (s3h_md5_batch_routed): ((n, 4) uint32, taken)."""
    arrs, ptrs, lens = _host_parts(parts)
    out = np.zeros((len(arrs), 4), dtype=np.uint32)
    taken = ctypes.c_int(-1)
    check(lib().s3h_md5_batch_routed(ptrs, _p64(lens), len(arrs), out.ctypes.data, ndevices,
                                     _native.ROUTE_IDS[route], ctypes.byref(taken)))
    return out, _native.ROUTE_NAMES[taken.value]


def sha256_md5_batch_routed(parts: Sequence, ndevices: int = 0,
                            route: str = "auto") -> tuple[np.ndarray, np.ndarray, str]:
    """x-amz-content-sha256 AND Content-MD5 of host parts on a route -- "gpu" (one grid, one
    PCIe pass: sha256_md5_batch_host), "cpu" (both digests per part in one pass over memory),
    "split" or "auto" (priced with the dual rates) -- s3h_sha256_md5_batch_routed.  Returns
    ((n, 8) SHA-256 words, (n, 4) MD5 words, route taken)."""
    arrs, ptrs, lens = _host_parts(parts)
    sha = np.zeros((len(arrs), DIGEST_WORDS), dtype=np.uint32)
    m5 = np.zeros((len(arrs), 4), dtype=np.uint32)
    taken = ctypes.c_int(-1)
    check(lib().s3h_sha256_md5_batch_routed(ptrs, _p64(lens), len(arrs), sha.ctypes.data,
                                            m5.ctypes.data, ndevices, _native.ROUTE_IDS[route],
                                            ctypes.byref(taken)))
    return sha, m5, _native.ROUTE_NAMES[taken.value]


def sha256_md5_file_parts_routed(path: str, offsets, lengths, ndevices: int = 0,
                                 route: str = "auto") -> tuple[np.ndarray, np.ndarray, str]:
    """Both digests of file ranges on a route (s3h_sha256_md5_file_parts_routed)."""
    offs, lens = _u64(offsets), _u64(lengths)
    if offs.shape != lens.shape or offs.ndim != 1 or offs.size == 0:
        raise ValueError("offsets and lengths must be 1-D, equal length and non-empty")
    sha = np.zeros((offs.size, DIGEST_WORDS), dtype=np.uint32)
    m5 = np.zeros((offs.size, 4), dtype=np.uint32)
    taken = ctypes.c_int(-1)
    check(lib().s3h_sha256_md5_file_parts_routed(os.fsencode(path), _p64(offs), _p64(lens),
                                                 offs.size, sha.ctypes.data, m5.ctypes.data,
                                                 ndevices, _native.ROUTE_IDS[route],
                                                 ctypes.byref(taken)))
    return sha, m5, _native.ROUTE_NAMES[taken.value]


def md5_file_parts(path: str, offsets, lengths, ndevices: int = 0, slice_bytes: int = 0) -> np.ndarray:
    """Content-MD5 of file ranges on the GPU (s3h_md5_file_parts): (n, 4) uint32."""
    offs, lens = _u64(offsets), _u64(lengths)
    if offs.shape != lens.shape or offs.ndim != 1 or offs.size == 0:
        raise ValueError("offsets and lengths must be 1-D, equal length and non-empty")
    out = np.zeros((offs.size, 4), dtype=np.uint32)
    check(lib().s3h_md5_file_parts(os.fsencode(path), _p64(offs), _p64(lens), offs.size,
                                   out.ctypes.data, ndevices, slice_bytes))
    return out


def route_rates() -> dict:
    """The whole routing model -- per digest set (index 0 SHA-256, 1 MD5, 2 both) the one-thread
    and all-threads CPU rates and the GPU chain rate, H2D / staging rates, call cost, the
    observed GPU / CPU factors, measurement and divergence counters (s3h_route_rates; measures
    what is missing).  Lists for the per-digest-set arrays."""
    r = _native.RouteRates()
    r.size = ctypes.sizeof(r)
    check(lib().s3h_route_rates(ctypes.byref(r)))
    out = {}
    for f, _ in r._fields_:
        v = getattr(r, f)
        out[f] = list(v) if isinstance(v, ctypes.Array) else v
    return out


def route_choose(lengths, rates: dict, digests: str = "sha256", ndevices: int = 0,
                 source: str = "pinned") -> dict:
    """AUTO's decision under ``rates`` (route_rates()'s dict, possibly edited; pure host
    arithmetic, s3h_route_choose): route, gpu_s, cpu_s, split_s, cpu_parts, stage_threads."""
    r = _native.RouteRates()
    for f, _ in r._fields_:
        if f in rates:
            v = rates[f]
            if isinstance(v, (list, tuple)):
                arr = getattr(r, f)
                for i, x in enumerate(v):
                    arr[i] = x
            else:
                setattr(r, f, v)
    r.size = ctypes.sizeof(r)
    lens = _u64(lengths)
    c = _native.RouteChoice()
    check(lib().s3h_route_choose(ctypes.byref(r), _native.DIGESTS_IDS[digests], _p64(lens), lens.size,
                                 ndevices, _native.SOURCE_IDS[source], ctypes.byref(c)))
    return {"route": _native.ROUTE_NAMES[c.route], "gpu_s": c.gpu_s, "cpu_s": c.cpu_s,
            "split_s": c.split_s, "cpu_parts": c.cpu_parts, "stage_threads": c.stage_threads}


def route_device_rates(device: int, digests: str = "sha256") -> tuple[float, float]:
    """(lone-chain bytes/s, pinned H2D bytes/s) of one device (s3h_route_device_rates)."""
    ch, h = ctypes.c_double(), ctypes.c_double()
    check(lib().s3h_route_device_rates(device, _native.DIGESTS_IDS[digests], ctypes.byref(ch),
                                       ctypes.byref(h)))
    return ch.value, h.value


def route_refresh_calls(calls: int) -> int:
    """Re-measure the routing model every ``calls`` AUTO/SPLIT calls (0: only on divergence);
    returns the previous setting (s3h_route_refresh_calls)."""
    prev = ctypes.c_int(0)
    check(lib().s3h_route_refresh_calls(int(calls), ctypes.byref(prev)))
    return prev.value


def route_scale(rate: str, factor: float) -> None:
    """Test hook: multiply one measured rate ("chain", "h2d", "cpu", "staged") by ``factor``
    until the model is next measured (s3h_route_scale)."""
    check(lib().s3h_route_scale(_native.RATE_IDS[rate], float(factor)))


def host_plan(pci_bus_ids, affinity: str | None = None, cpu_quota: float = -1.0) -> dict:
    """The host path's thread plan for a call over the devices at ``pci_bus_ids`` (None
    entries: no NUMA record) -- per-device staging threads, bind node and CPUs, split-route
    thread shares, oversubscription flags -- with the CPUs of ``affinity`` (a cpulist; None:
    this process) under a ``cpu_quota`` (0: none; < 0: this process's cgroup): s3h_host_plan,
    pure host arithmetic over sysfs (S3H_SYSFS_ROOT)."""
    n = len(pci_bus_ids)
    ids = (ctypes.c_char_p * n)(*[None if b is None else b.encode() for b in pci_bus_ids])
    plan = _native.HostPlan()
    devs = (_native.HostPlanDevice * n)()
    check(lib().s3h_host_plan(ids, n, None if affinity is None else affinity.encode(),
                              float(cpu_quota), ctypes.byref(plan), devs))
    out = {f: getattr(plan, f) for f, _ in plan._fields_}
    out["per_device"] = [{f: getattr(d, f) for f, _ in d._fields_} for d in devs]
    return out


def host_threads(ndevices: int = 1) -> tuple[int, int]:
    """(staging threads per device when ``ndevices`` device shards run at once, CPUs this
    process may use: affinity capped by the cgroup quota) -- s3h_host_threads."""
    cpus = ctypes.c_int(0)
    per = lib().s3h_host_threads(ndevices, ctypes.byref(cpus))
    return per, cpus.value


def pci_numa(pci_bus_id: str) -> dict:
    """sysfs NUMA record of a PCI function (s3h_pci_numa; no GPU needed): node, local CPU
    list and how many of those CPUs this thread may run on."""
    node, usable = ctypes.c_int(-1), ctypes.c_int(0)
    buf = ctypes.create_string_buffer(4096)
    check(lib().s3h_pci_numa(pci_bus_id.encode(), ctypes.byref(node), buf, len(buf),
                             ctypes.byref(usable)))
    return {"node": node.value, "local_cpulist": buf.value.decode(), "usable_cpus": usable.value}


def device_numa(device: int) -> dict:
    """NUMA node and local CPU list of HIP device ``device`` (s3h_device_numa_node)."""
    node = ctypes.c_int(-1)
    buf = ctypes.create_string_buffer(4096)
    check(lib().s3h_device_numa_node(device, ctypes.byref(node), buf, len(buf)))
    return {"node": node.value, "local_cpulist": buf.value.decode()}


def host_numa(mode) -> int:
    """Set the host path's placement policy -- "local" (each device's node, the default), "off"
    (runtime placement, unbound threads) or a node number -- and return the previous mode
    (-1 local, -2 off, else a node): s3h_host_numa."""
    m = {"local": _native.NUMA_LOCAL, "off": _native.NUMA_OFF}.get(mode, mode)
    prev = ctypes.c_int(0)
    check(lib().s3h_host_numa(int(m), ctypes.byref(prev)))
    return prev.value


def host_numa_info(device: int) -> dict:
    """Where the host path places device ``device``'s staging and copy threads, and what its
    cached context holds (s3h_host_numa_info)."""
    info = _native.HostNuma()
    check(lib().s3h_host_numa_info(device, ctypes.byref(info)))
    return {f: getattr(info, f) for f, _ in info._fields_}


def mem_node(buf) -> int:
    """NUMA node of the page holding the start of ``buf`` (numpy array, CPU torch tensor or an
    address): s3h_mem_node."""
    addr = buf if isinstance(buf, int) else (buf.data_ptr() if hasattr(buf, "data_ptr")
                                             else _as_bytes(buf).ctypes.data)
    node = ctypes.c_int(-1)
    check(lib().s3h_mem_node(ctypes.c_void_p(addr), ctypes.byref(node)))
    return node.value


class PinnedBuffer:
    """Pinned host memory on a NUMA node (s3h_host_alloc; node -1 = the runtime's placement),
    e.g. an uploader's read buffer on its device's node.  ``array`` is a uint8 numpy view (it
    keeps the buffer alive); the memory is freed when the last view is gone or on close()."""

    def __init__(self, nbytes: int, node: int = -1, strict: bool = False):
        import weakref
        p = ctypes.c_void_p()
        flags = _native.HOST_ALLOC_STRICT if strict else 0
        check(lib().s3h_host_alloc_ex(int(node), int(nbytes), flags, ctypes.byref(p)))
        self.ptr, self.nbytes, self.node = p.value, int(nbytes), int(node)
        raw = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
        # freed once the ctypes array -- held by this object and by every numpy view -- is gone
        self._free = weakref.finalize(raw, lib().s3h_host_free, ctypes.c_void_p(self.ptr))
        self.array = np.frombuffer(raw, dtype=np.uint8)

    def close(self) -> None:
        """Free now (no view of ``array`` may be used afterwards)."""
        self.array = None
        self._free()


def dual_layout(lengths, cus: int = 256) -> tuple[int, bool]:
    """(skew groups of the SHA-256 + MD5 mixed grid, MD5 apart?) for a batch of ``lengths`` on
    a device of ``cus`` CUs -- the rule a plan applies, on the host (s3h_dual_layout)."""
    lens = _u64(lengths)
    solo, apart = ctypes.c_uint32(), ctypes.c_int()
    check(lib().s3h_dual_layout(_p64(lens), lens.size, cus, ctypes.byref(solo), ctypes.byref(apart)))
    return solo.value, bool(apart.value)


def kernel_policy(policy: str) -> str:
    """AUTO's kernel policy for plans created afterwards -- "throughput" (skews for 4,097 -
    32 x CUs parts), "efficiency" (skewp there: ~5 % slower, ~36 % fewer joules per GiB) or
    "power" (the default: skews only when the board's power cap lets it hold its clock) --
    returns the previous one (s3h_kernel_policy)."""
    prev = ctypes.c_int(0)
    check(lib().s3h_kernel_policy(_native.POLICY_IDS[policy], ctypes.byref(prev)))
    return _native.POLICY_NAMES[prev.value]


def device_power_cap(device: int = 0) -> float:
    """Board power cap of ``device`` in watts as the "power" kernel policy reads it (sysfs hwmon
    power1_cap; 0.0 when the platform does not say): s3h_device_power_cap."""
    w = ctypes.c_double(0)
    check(lib().s3h_device_power_cap(device, ctypes.byref(w)))
    return w.value


def pci_power_cap(pci_bus_id: str) -> float:
    """Board power cap in watts of the PCI function (sysfs hwmon power1_cap; 0.0 when absent;
    no GPU needed): s3h_pci_power_cap."""
    w = ctypes.c_double(0)
    check(lib().s3h_pci_power_cap(pci_bus_id.encode(), ctypes.byref(w)))
    return w.value


def trim() -> None:
    """Free the host path's cached per-device buffers (HBM ring, pinned staging, plans):
    s3h_trim.  A process that shares the GPU with other work calls this when it is done."""
    check(lib().s3h_trim())


def generate_parts(data, offsets, lengths, part_ids, seed: int, stream=None) -> None:
    """Fill parts of device tensor ``data`` with generator G(seed, part_id, length)."""
    offs, lens, ids = _u64(offsets), _u64(lengths), _u64(part_ids)
    dev = data.device.index
    for s in range(0, offs.size, 65535):
        e = min(offs.size, s + 65535)
        check(lib().s3h_generate_parts(dev, ctypes.c_void_p(data.data_ptr()), _p64(offs[s:e]),
                                       _p64(lens[s:e]), _p64(ids[s:e]), e - s, seed,
                                       ctypes.c_void_p(_stream_handle(stream))))


# ------------------------------------------------------------------ CPU drop-in (lib/hash)
def sha256(data: bytes) -> np.ndarray:
    """lib/hash sha256::sha256 (CPU, single message): 8 words, hash[i] = bswap32(H_i)."""
    b = bytes(data)
    out = np.zeros(DIGEST_WORDS, dtype=np.uint32)
    lib().s3h_cpu_sha256(b, len(b), out.ctypes.data)
    return out


def md5(data: bytes) -> np.ndarray:
    """lib/hash md5 drop-in (CPU, single message, padded): 4 words, LE digest bytes."""
    b = bytes(data)
    out = np.zeros(4, dtype=np.uint32)
    lib().s3h_cpu_md5(b, len(b), out.ctypes.data)
    return out


def hmac256(data: bytes, key: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    d, k = bytes(data), bytes(key)
    lib().s3h_cpu_hmac256(d, len(d), k, len(k), out)
    return out.raw


def hash_to_text(words) -> str:
    """sha256::hash_to_text / md5::hash_to_text: lowercase hex of the digest bytes in memory."""
    return np.ascontiguousarray(words, dtype=np.uint32).reshape(-1).tobytes().hex()


def digests_to_text(words, nwords: int = DIGEST_WORDS) -> list[str]:
    w = np.ascontiguousarray(words).view(np.uint32).reshape(-1, nwords)
    return [row.tobytes().hex() for row in w]


def cpu_backend() -> str:
    return lib().s3h_cpu_backend().decode()
