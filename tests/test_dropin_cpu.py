"""libs3hash.so on the CPU: it loads, exports every C-ABI symbol of include/s3hash.h and the
lib/hash C++ drop-in symbols, and its single-message sha256/hmac256 match the golden
vectors (no GPU needed; no compute call reaches HIP here)."""
import ctypes
import os
import sys
import hashlib
import subprocess

import numpy as np
import pytest

import s3client_amd as s3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from s3client_amd import _native


def test_library_exports_every_symbol():
    L = _native.lib()
    for name in _native.C_ABI_SYMBOLS + _native.CXX_DROPIN_SYMBOLS:
        assert hasattr(L, name), name


def test_header_declares_exactly_the_exported_c_abi():
    import os, re
    hdr = open(os.path.join(os.path.dirname(_native.__file__), "..", "include", "s3hash.h")).read()
    declared = set(re.findall(r"\b(s3h_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(_native.C_ABI_SYMBOLS)


def test_nm_shows_reference_mangled_names():
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for name in _native.CXX_DROPIN_SYMBOLS:
        assert f" T {name}" in out, name


@pytest.mark.parametrize("backend", ["default", "scalar"])
def test_cpu_sha256_golden(golden, oracle, backend, monkeypatch):
    if backend == "scalar":
        # the scalar fallback is chosen at load time: run it in a child process
        code = ("import json,sys;import s3client_amd as s;from tests.oracle_lib import Oracle;"
                "o=Oracle();g=json.load(open('tests/golden/sha256_golden.json'));"
                "big=o.generate(7,max(e['L'] for e in g['edge']));"
                "bad=[e['L'] for e in g['edge'] if s.hash_to_text(s.sha256(big[:e['L']]))!=e['digest']];"
                "assert s.cpu_backend()=='scalar';print(bad);sys.exit(1 if bad else 0)")
        r = subprocess.run(["python", "-c", code], env={**__import__("os").environ,
                           "S3H_CPU_SCALAR": "1"}, capture_output=True, text=True,
                           cwd=_native._HERE + "/..")
        assert r.returncode == 0, r.stdout + r.stderr
        return
    for k in golden["kat"]:
        assert s3.hash_to_text(s3.sha256(k["ascii"].encode())) == k["digest"]
    big = oracle.generate(7, max(e["L"] for e in golden["edge"]))
    for e in golden["edge"]:
        assert s3.hash_to_text(s3.sha256(big[:e["L"]])) == e["digest"], e["L"]


def test_cpu_hmac_golden(golden):
    for h in golden["hmac"]:
        assert s3.hmac256(bytes.fromhex(h["msg"]), bytes.fromhex(h["key"])).hex() == h["mac"]


def test_hmac_long_key_is_rfc2104():
    key, msg = bytes(range(100)), b"x" * 10  # key > 64, len(msg) != len(key)
    import hmac
    assert s3.hmac256(msg, key) == hmac.new(key, msg, hashlib.sha256).digest()


def test_hash_to_text_c_view():
    w = s3.sha256(b"abc")
    buf = ctypes.create_string_buffer(65)
    _native.lib().s3h_hash_to_text(w.ctypes.data, buf)
    assert buf.value.decode() == hashlib.sha256(b"abc").hexdigest() == s3.hash_to_text(w)


def test_gpu_entry_points_fail_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(s3.S3HashError) as ei:
        s3.Plan([0], [10])
    assert ei.value.code in (_native.S3H_ENODEV, _native.S3H_EHIP)
    with pytest.raises(s3.S3HashError):
        s3.sha256_batch_host([b"abc"])


def test_cpu_md5_golden(golden, oracle):
    import hashlib
    md = golden["md5"]
    big = oracle.generate(7, max(e["L"] for e in md["edge"]))
    for e in md["edge"]:
        assert s3.hash_to_text(s3.md5(big[:e["L"]])) == e["digest"], e["L"]
    assert s3.hash_to_text(s3.md5(b"")) == hashlib.md5(b"").hexdigest()


def test_multipart_etag_golden(golden):
    words = [np.frombuffer(bytes.fromhex(p["digest"]), dtype=np.uint32) for p in golden["md5"]["transfer"]]
    assert s3.multipart_etag(np.stack(words)) == golden["md5"]["transfer_etag"]  # s3h_multipart_etag
    with pytest.raises(s3.S3HashError):
        s3.multipart_etag(np.zeros((0, 4), dtype=np.uint32))


def test_kernel_isa_counts_match_the_built_code_object(tmp_path):
    """bench.py's `issue` field divides cycles by s3client_amd/kernel_isa_counts.json; that file
    must be what tools/isa_counts.py derives from the code object `make` just built."""
    import json
    import subprocess
    out = tmp_path / "counts.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_counts.py"), _native.LIB_PATH,
                    str(out)], check=True, capture_output=True)
    with open(out) as f:
        fresh = json.load(f)
    with open(os.path.join(ROOT, "s3client_amd", "kernel_isa_counts.json")) as f:
        shipped = json.load(f)
    # the kernel code hashes bench.py matches PMC profiles against are the built library's
    assert fresh["code_hash"] == shipped["code_hash"] and len(shipped["code_hash"]) >= 8
    assert fresh == shipped
    k = shipped["kernels"]
    assert 540 < k["skew"]["instr_per_block"] < 550 and 600 < k["skewp"]["instr_per_block"] < 615
    assert k["skew"]["per_block"]["lds"] == 16.0
    # the shared-SIMD kernel's consumer is the flag-synchronised skew consumer (the producer
    # beside it runs on the same SIMD and is not in this loop)
    assert abs(k["skews"]["instr_per_block"] - k["skew_nc2"]["instr_per_block"]) < 1.0


# ------------------------------------------------------------------ size-aware routing
_MODEL = dict(cpu_bytes_per_s=1.5e9, chain_bytes_per_s=69e6, h2d_bytes_per_s=50e9, call_s=2e-4,
              cpu_threads=16, devices=1)


def test_route_estimate_crossover():
    """AUTO's model (s3h_route_estimate): a few 8 MiB parts finish first on 16 SHA-NI threads
    (one GPU chain needs 8 MiB / 69 MB/s = 0.12 s), 1,024 of them on the GPU (PCIe-bound
    0.17 s vs 0.36 s on the CPU); one thread per part at most; bad models are rejected."""
    r, g, c = s3.route_estimate([8 << 20] * 128, _MODEL)
    assert r == "cpu" and abs(g - (2e-4 + (8 << 20) / 69e6)) < 1e-9 and c < g
    r, g, c = s3.route_estimate([8 << 20] * 1024, _MODEL)
    assert r == "gpu" and abs(g - (2e-4 + 1024 * (8 << 20) / 50e9)) < 1e-9 and c > g
    _, _, c1 = s3.route_estimate([8 << 20] * 2, _MODEL)
    assert abs(c1 - (8 << 20) / 1.5e9) < 1e-12  # two parts: two threads, not sixteen
    _, g2, _ = s3.route_estimate([8 << 20] * 1024, {**_MODEL, "devices": 2}, ndevices=0)
    assert abs(g2 - (2e-4 + max((8 << 20) / 69e6, 512 * (8 << 20) / 50e9))) < 1e-9  # per device
    with pytest.raises(s3.S3HashError):
        s3.route_estimate([1], {**_MODEL, "chain_bytes_per_s": 0.0})


def test_route_estimate_measured_team_rate_and_schedule():
    """Round 5 model: the CPU route on k threads runs at min(k x one-thread rate, the measured
    all-threads rate), parts are scheduled longest first (24 equal parts on 16 threads take two
    part-times, not 1.5), and pageable parts feed the GPU at min(h2d, staged)."""
    M = {**_MODEL, "cpu_all_bytes_per_s": 16e9, "staged_bytes_per_s": 30e9}
    P = 8 << 20
    _, _, c = s3.route_estimate([P] * 4, M)  # 4 threads: 6e9 < 16e9, per thread 1.5e9
    assert abs(c - P / 1.5e9) < 1e-12
    _, _, c = s3.route_estimate([P] * 16, M)  # 16 threads share 16e9: 1e9 each
    assert abs(c - P / 1e9) < 1e-12
    _, _, c = s3.route_estimate([P] * 24, M)  # longest first: 8 threads hash two parts
    assert abs(c - 2 * P / 1e9) < 1e-12
    _, _, c = s3.route_estimate([3 * P, P, P, P], {**M, "cpu_threads": 2})  # 3P | P+P+P
    assert abs(c - 3 * P / 1.5e9) < 1e-12
    _, g_pin, _ = s3.route_estimate([P] * 1024, M, source="pinned")
    _, g_pag, _ = s3.route_estimate([P] * 1024, M, source="pageable")
    _, g_file, _ = s3.route_estimate([P] * 1024, M, source="file")
    assert abs(g_pin - (2e-4 + 1024 * P / 50e9)) < 1e-9
    assert abs(g_pag - (2e-4 + 1024 * P / 30e9)) < 1e-9 and g_file == g_pag
    # with the linear estimate 1,024 parts looked 1.5x faster on the CPU than they are
    r_lin, _, c_lin = s3.route_estimate([P] * 1024, _MODEL)
    r, _, c = s3.route_estimate([P] * 1024, M)
    assert r_lin == r == "gpu" and abs(c / c_lin - 24e9 / 16e9) < 1e-9
    assert s3._native.lib().s3h_route_estimate_ex(None, None, 1, 0, 3, None, None) == -1


def test_cpu_route_batch_vs_oracle(oracle):
    """S3H_ROUTE_CPU: the lib/hash drop-in on host threads, longest part first, bit-exact vs
    the oracle (empty parts, every tail length)."""
    rng = np.random.default_rng(77)
    lens = np.concatenate([[0, 1, 55, 56, 63, 64, 65, 119, 120, (4 << 20) + 1, 9 << 20],
                           rng.integers(0, 300000, 40)])
    data = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in lens]
    got, taken = s3.sha256_batch_routed(data, route="cpu")
    assert taken == "cpu"
    assert np.array_equal(got, np.stack([oracle.sha256(d.tobytes()) for d in data]))


def test_cpu_route_file_parts_vs_oracle(oracle, tmp_path):
    """The same for (file, offset, size) ranges: pread in 4 MiB chunks, streamed, the last chunk
    padded with the part's total length -- ranges straddling chunk edges, empty, misaligned."""
    rng = np.random.default_rng(78)
    blob = rng.integers(0, 256, (13 << 20) + 333, dtype=np.uint8)
    path = tmp_path / "object.bin"
    blob.tofile(path)
    ranges = [(0, 0), (0, 4 << 20), (1, (4 << 20) + 1), (3, (8 << 20) - 1), (7, (12 << 20) + 64),
              (blob.size - 1, 1), (12345, 55), (777, 0), (5, blob.size - 5)]
    offs = [o for o, _ in ranges]
    lens = [L for _, L in ranges]
    got, taken = s3.sha256_file_parts_routed(str(path), offs, lens, route="cpu")
    assert taken == "cpu"
    want = np.stack([oracle.sha256(blob[o:o + L].tobytes()) for o, L in ranges])
    assert np.array_equal(got, want)
    with pytest.raises(s3.S3HashError):  # a range past the end of the file
        s3.sha256_file_parts_routed(str(path), [blob.size - 10], [11], route="cpu")
    with pytest.raises(s3.S3HashError):  # offset + length wraps past 2^64
        s3.sha256_file_parts_routed(str(path), [2**64 - 1], [2], route="cpu")
    with pytest.raises(s3.S3HashError):
        s3.sha256_file_parts_routed(str(tmp_path / "missing"), [0], [1], route="cpu")


def test_route_auto_is_not_a_fallback():
    """AUTO chooses between the GPU and the CPU drop-in; with no GPU it fails (S3H_ENODEV)
    instead of running everything on the CPU.  An unknown route is rejected."""
    with pytest.raises(s3.S3HashError) as e:
        s3.sha256_batch_routed([b"abc"], route="auto")
    assert e.value.code == -2
    with pytest.raises(s3.S3HashError) as e:
        s3.sha256_batch_routed([b"abc", b"de"], route="split")
    assert e.value.code == -2
    exp = np.zeros((2, 8), dtype=np.uint32)
    with pytest.raises(s3.S3HashError) as e:
        s3.verify_batch_routed([b"abc", b"de"], exp, route="auto")
    assert e.value.code == -2
    with pytest.raises(s3.S3HashError) as e:  # MD5 verifies on the GPU route only
        s3.verify_batch_routed([b"abc", b"de"], exp[:, :4], algo="md5", route="split")
    assert e.value.code == -1
    with pytest.raises(s3.S3HashError) as e:
        s3.route_model()
    assert e.value.code == -2
    from s3client_amd import _native
    rc = _native.lib().s3h_sha256_batch_routed(None, None, 0, None, 0, 7, None)
    assert rc == -1
