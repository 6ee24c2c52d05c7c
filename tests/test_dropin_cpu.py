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
    assert fresh == shipped
    k = shipped["kernels"]
    assert 540 < k["skew"]["instr_per_block"] < 550 and 600 < k["skewp"]["instr_per_block"] < 615
    assert k["skew"]["per_block"]["lds"] == 16.0
    # the shared-SIMD kernel's consumer is the flag-synchronised skew consumer (the producer
    # beside it runs on the same SIMD and is not in this loop)
    assert abs(k["skews"]["instr_per_block"] - k["skew_nc2"]["instr_per_block"]) < 1.0
