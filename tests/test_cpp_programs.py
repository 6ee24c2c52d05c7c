"""C++ programs linked against libs3hash.so the way the reference's callers link lib/hash:
the signer KATs of config 1 (test/sign-test.cpp, test/presign-url-test.cpp) through the
drop-in, and the lib/hash drop-in known-answer tests.  `--gpu` adds the batched C++ API."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "cpp", "build")


@pytest.fixture(scope="module")
def programs():
    subprocess.run(["make", "-C", ROOT, "cpptests"], check=True, capture_output=True)
    return BUILD


def _run(path, *args):
    r = subprocess.run([path, *args], capture_output=True, text=True, timeout=300)
    rows = [l.split(",") for l in r.stdout.strip().splitlines()]
    return r.returncode, rows


def test_sign_kats(programs):
    rc, rows = _run(os.path.join(programs, "sign_test"))
    assert rc == 0 and rows and all(r[2] == "1" for r in rows), rows
    assert {r[1] for r in rows} >= {"Sign request", "Presign URL", "Sign payload request"}


def test_dropin_kats(programs):
    rc, rows = _run(os.path.join(programs, "dropin_test"))
    assert rc == 0 and len(rows) >= 12 and all(r[2] == "1" for r in rows), rows


@pytest.mark.gpu
def test_dropin_gpu_batch(programs):
    rc, rows = _run(os.path.join(programs, "dropin_test"), "--gpu")
    assert rc == 0, rows
    got = {r[1]: r[2] for r in rows}
    assert got["gpu batch payload_hashes"] == "1" and got["gpu stream_batch"] == "1", rows
    assert got["gpu sha256_md5_batch"] == "1" and got["gpu concurrent jobs"] == "1", rows
    assert got["gpu routed payload_hashes"] == "1", rows


def _xfer_file(tmp_path, golden):
    import numpy as np
    t = golden["transfer"]
    p = tmp_path / "xfer.bin"
    (np.arange(t["size"], dtype=np.uint64) % 128).astype(np.uint8).tofile(p)
    return str(p), t


def _parse_parts(stdout):
    lines = [l for l in stdout.splitlines() if l and not l.startswith("#")]
    assert lines[0] == "part,job,offset,size,sha256"
    return [l.split(",") for l in lines[1:]]


def test_upload_counterpart_cpu(programs, tmp_path, golden):
    """apps/s3_upload_hash.cpp with the CPU drop-in: the transfer test's 3 jobs x 2 parts."""
    path, t = _xfer_file(tmp_path, golden)
    app = os.path.join(ROOT, "apps", "build", "s3-upload-hash")
    r = subprocess.run([app, "-f", path, "-j", "3", "-n", "2", "--cpu", "--print-headers"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = _parse_parts(r.stdout)
    assert [(int(x[2]), int(x[3]), x[4]) for x in rows] == \
        [(p["offset"], p["size"], p["digest"]) for p in t["parts"]]
    heads = [l for l in r.stdout.splitlines() if " x-amz-content-sha256: " in l]
    assert len(heads) == 6 and "UNSIGNED-PAYLOAD" not in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["file", "mmap", "memory"])
@pytest.mark.parametrize("per_job", [False, True])
def test_upload_counterpart_gpu(programs, tmp_path, golden, source, per_job):
    """UploadFile (file ranges / mmap) and UploadData (memory buffer) counterparts, one batch
    call or one concurrent call per job: the transfer test's 3 jobs x 2 parts vs lib/hash."""
    path, t = _xfer_file(tmp_path, golden)
    app = os.path.join(ROOT, "apps", "build", "s3-upload-hash")
    cmd = [app, "-f", path, "-j", "3", "-n", "2", "--verify", "--source", source, "--print-headers"]
    r = subprocess.run(cmd + (["--per-job"] if per_job else []), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    rows = _parse_parts(r.stdout)
    assert [x[4] for x in rows] == [p["digest"] for p in t["parts"]]
    heads = [l for l in r.stdout.splitlines() if " x-amz-content-sha256: " in l]
    assert [h.split(": ")[-1] for h in heads] == [p["digest"] for p in t["parts"]]


@pytest.mark.gpu
@pytest.mark.parametrize("jobs,ppj", [(1, 3), (2, 1)])
def test_upload_counterpart_memory_multipart(programs, tmp_path, golden, jobs, ppj):
    """UploadData geometry of test/api/multipart-upload-test.cpp:47-54 (19,000,000 iota bytes in
    3 or 2 chunks): the memory path forwards each part's digest into its signature (the
    reference's DoUploadPart drops it, multipart_upload.cpp:131-136)."""
    import numpy as np
    mp = golden["multipart"]
    path = tmp_path / "mp.bin"
    (np.arange(mp["size"], dtype=np.uint64) % 256).astype(np.uint8).tofile(path)
    app = os.path.join(ROOT, "apps", "build", "s3-upload-hash")
    r = subprocess.run([app, "-f", str(path), "-j", str(jobs), "-n", str(ppj), "--source", "memory",
                        "--per-job", "--print-headers"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rows = _parse_parts(r.stdout)
    want = [p for p in mp["parts"] if p["chunks"] == jobs * ppj]
    assert [(int(x[2]), int(x[3]), x[4]) for x in rows] == [(p["offset"], p["size"], p["digest"]) for p in want]
    assert "UNSIGNED-PAYLOAD" not in r.stdout


def _start_mock(*args):
    """tests/s3_mock_server.py on a free loopback port: checks every PUT body's SHA-256 against
    x-amz-content-sha256 and verifies its SigV4 signature (config 5's endpoint; MinIO absent).
    Returns (process, url, stats())."""
    import json
    import sys
    import time
    import urllib.request
    proc = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "s3_mock_server.py"),
                             "--port", "0", *args], stdout=subprocess.PIPE, text=True)
    url = f"http://127.0.0.1:{int(proc.stdout.readline())}"

    def stats():
        for _ in range(50):
            try:
                with urllib.request.urlopen(url + "/stats", timeout=5) as r:
                    return json.loads(r.read())
            except OSError:
                time.sleep(0.1)
        raise RuntimeError("mock S3 server not answering")
    return proc, url, stats


@pytest.fixture
def s3_mock():
    proc, url, stats = _start_mock()
    try:
        yield url, stats
    finally:
        proc.kill()
        proc.wait()


def _upload(app_args, url, tmp_path, golden):
    path, t = _xfer_file(tmp_path, golden)
    app = os.path.join(ROOT, "apps", "build", "s3-upload-hash")
    r = subprocess.run([app, "-f", path, "-j", "3", "-n", "2", "--send", "--endpoint", url,
                        *app_args], capture_output=True, text=True, timeout=300)
    return r, t


def test_upload_send_loopback_cpu(programs, tmp_path, golden, s3_mock):
    """Config 5's path without MinIO: the CPU drop-in hashes the transfer test's 3 jobs x 2 parts
    and each job PUTs its parts with the digest signed into x-amz-content-sha256; the loopback
    server accepts all six (body SHA-256 and signature verified), and rejects every part signed
    with another secret."""
    url, stats = s3_mock
    for source in ("file", "memory"):
        r, t = _upload(["--cpu", "--source", source], url, tmp_path, golden)
        assert r.returncode == 0, r.stderr
        assert [x[4] for x in _parse_parts(r.stdout)] == [p["digest"] for p in t["parts"]]
    s = stats()
    assert s["parts"] == 12 and s["bytes"] == 2 * t["size"], s
    assert s["bad_hash"] == 0 and s["bad_signature"] == 0, s
    r, _ = _upload(["--cpu", "--secret", "WRONG"], url, tmp_path, golden)
    assert r.returncode != 0 and "6 of 6 PUTs not 200" in r.stderr, r.stderr
    assert stats()["bad_signature"] == 6


def test_upload_send_endpoint_down(programs, tmp_path, golden):
    """No server listening: every PUT fails, the app reports it and exits non-zero (no hang,
    no SIGPIPE)."""
    import socket
    with socket.socket() as sk:  # a port that was free a moment ago and has no listener
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r, _ = _upload(["--cpu"], f"http://127.0.0.1:{port}", tmp_path, golden)
    assert r.returncode == 1 and "6 of 6 PUTs not 200" in r.stderr, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("source,per_job", [("file", False), ("mmap", True), ("memory", True)])
def test_upload_send_loopback_gpu(programs, tmp_path, golden, s3_mock, source, per_job):
    """The same upload with the GPU batch path (H2D included): one call, or one concurrent call
    per job thread before it PUTs its parts; every part accepted by the verifying server."""
    url, stats = s3_mock
    r, t = _upload(["--source", source] + (["--per-job"] if per_job else []), url, tmp_path, golden)
    assert r.returncode == 0, r.stderr
    assert [x[4] for x in _parse_parts(r.stdout)] == [p["digest"] for p in t["parts"]]
    s = stats()
    assert s["parts"] == 6 and s["bad_hash"] == 0 and s["bad_signature"] == 0, s


def test_upload_send_retries_and_endpoints(programs, tmp_path, golden):
    """upload.cpp's endpoint list and retries: jobs draw their endpoint at random from two
    servers (upload.cpp:94-95); one server answers every 3rd PUT with 503, and a failed part is
    signed and sent again while the shared --retries budget lasts (upload.cpp:55-87).  With no
    budget the failures surface."""
    servers = [_start_mock("--fail-every", "3"), _start_mock()]
    try:
        urls = ",".join(u for _, u, _ in servers)
        for _ in range(2):
            r, t = _upload(["--cpu", "--retries", "20"], urls, tmp_path, golden)
            assert r.returncode == 0, r.stderr
        st = [f() for _, _, f in servers]
        assert sum(x["parts"] for x in st) == 12, st
        assert all(x["bad_hash"] == 0 and x["bad_signature"] == 0 for x in st), st
        r, _ = _upload(["--cpu", "--retries", "0"], servers[0][1], tmp_path, golden)
        assert r.returncode == 1 and "2 of 6 PUTs not 200" in r.stderr, r.stderr
    finally:
        for p, _, _ in servers:
            p.kill()
            p.wait()


def test_upload_send_content_md5_cpu(programs, tmp_path, golden, s3_mock):
    """--content-md5: each part also carries Content-MD5 (base64 of md5::md5 of the part); the
    endpoint checks it against the body (400 BadDigest otherwise) besides the SHA-256 and the
    signature."""
    url, stats = s3_mock
    r, t = _upload(["--cpu", "--content-md5"], url, tmp_path, golden)
    assert r.returncode == 0, r.stderr
    s = stats()
    assert s["parts"] == 6 and s["md5_checked"] == 6 and s["bad_md5"] == 0, s


@pytest.mark.gpu
@pytest.mark.parametrize("source,per_job", [("file", True), ("memory", False)])
def test_upload_send_content_md5_gpu(programs, tmp_path, golden, s3_mock, source, per_job):
    """The same with both digests from the GPU's dual pass (file ranges: one pread per slice
    for both; memory parts: one copy per slice for both)."""
    url, stats = s3_mock
    r, t = _upload(["--source", source, "--content-md5"] + (["--per-job"] if per_job else []),
                   url, tmp_path, golden)
    assert r.returncode == 0, r.stderr
    assert [x[4] for x in _parse_parts(r.stdout)] == [p["digest"] for p in t["parts"]]
    s = stats()
    assert s["parts"] == 6 and s["md5_checked"] == 6 and s["bad_md5"] == 0, s


def _etag_round(args, tmp_path, golden):
    """Upload of the transfer geometry to a correct endpoint (--content-md5: the multipart
    ETag printed equals the compiled reference's md5 golden) and to one that returns a
    non-MD5 ETag for part 4 -- as S3 does for SSE-KMS / SSE-C parts.  --content-md5 alone
    accepts it, as the reference does (DoUploadFilePart / DoUploadPart only require an ETag,
    multipart_upload.cpp:101-105, 138-143); --check-etag (with or without Content-MD5) fails
    the upload naming part 4, after its retries."""
    want = golden["md5"]["transfer_etag"]
    proc, url, stats = _start_mock()
    try:
        r, _ = _upload(args + ["--content-md5"], url, tmp_path, golden)
        assert r.returncode == 0, r.stderr
        assert f"multipart etag: {want}" in r.stderr, r.stderr
    finally:
        proc.kill()
        proc.wait()
    proc, url, stats = _start_mock("--wrong-etag-part", "4")
    try:
        r, _ = _upload(args + ["--content-md5", "--retries", "2"], url, tmp_path, golden)
        assert r.returncode == 0, r.stderr  # a non-MD5 ETag is an ETag
        assert stats()["wrong_etags"] == 1
        for extra in (["--content-md5"], []):
            r, _ = _upload(args + extra + ["--check-etag", "--retries", "2"], url, tmp_path, golden)
            assert r.returncode == 1, r.stderr
            assert "1 of 6 PUTs not 200" in r.stderr and "upload failed: part 4: ETag" in r.stderr, r.stderr
            assert "upload failed: part" not in r.stderr.replace("upload failed: part 4:", ""), r.stderr
        assert stats()["wrong_etags"] == 1 + 3 + 3  # each check: the first attempt and 2 retries
    finally:
        proc.kill()
        proc.wait()


def test_upload_etag_check_cpu(programs, tmp_path, golden):
    """UploadPart's ETag (multipart_upload.cpp:101-105, 138-143) checked against each part's MD5."""
    _etag_round(["--cpu"], tmp_path, golden)


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["file", "memory"])
def test_upload_etag_check_gpu(programs, tmp_path, golden, source):
    """The same with both digests from the GPU's dual pass: every returned ETag compared with
    the part's GPU MD5, a wrong one fails its part (named), the multipart ETag from the GPU
    MD5s equals the reference's."""
    _etag_round(["--source", source], tmp_path, golden)


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["cpu", "auto", "split"])
def test_upload_send_routed_gpu(programs, tmp_path, golden, s3_mock, route):
    """--route: the transfer test's 6 small parts hashed on the chosen route (auto: the
    measured model sends a batch this small to the CPU drop-in; split: the longest parts on
    the CPU beside the GPU) and PUT to the verifying endpoint; the digests are the lib/hash
    goldens either way."""
    url, stats = s3_mock
    r, t = _upload(["--route", route, "--source", "file"], url, tmp_path, golden)
    assert r.returncode == 0, r.stderr
    assert f"route {route} -> {'split' if route == 'split' else 'cpu'}" in r.stderr, r.stderr
    assert [x[4] for x in _parse_parts(r.stdout)] == [p["digest"] for p in t["parts"]]
    assert stats()["parts"] == 6


def test_upload_then_download_verify_cpu(programs, tmp_path, golden):
    """--get-verify: after the upload each job GETs its parts back by byte range (download.cpp
    geometry) from the storing endpoint and every part is checked against the digest it was
    uploaded with; a byte flipped in one GET response is caught."""
    proc, url, stats = _start_mock("--store")
    try:
        r, _ = _upload(["--cpu", "--get-verify"], url, tmp_path, golden)
        assert r.returncode == 0 and "0 GETs failed, 0 mismatches" in r.stderr, r.stderr
        assert stats()["gets"] == 6
    finally:
        proc.kill()
        proc.wait()
    proc, url, stats = _start_mock("--store", "--corrupt-get", "4")
    try:
        r, _ = _upload(["--cpu", "--get-verify"], url, tmp_path, golden)
        assert r.returncode == 1 and "0 GETs failed, 1 mismatches" in r.stderr, r.stderr
    finally:
        proc.kill()
        proc.wait()


@pytest.mark.gpu
def test_upload_then_download_verify_gpu(programs, tmp_path, golden):
    """The same round trip with the GPU: hash + PUT, ranged GETs, one s3h_verify_batch_host
    call over the downloaded parts (download verification)."""
    proc, url, stats = _start_mock("--store", "--corrupt-get", "2")
    try:
        r, _ = _upload(["--source", "memory", "--get-verify"], url, tmp_path, golden)
        assert r.returncode == 1 and "0 GETs failed, 1 mismatches" in r.stderr, r.stderr
        assert "GPU check" in r.stderr
    finally:
        proc.kill()
        proc.wait()


def _multipart_round(args, tmp_path, golden):
    """--multipart: the reference's whole UploadFile flow (upload.cpp:113-149) against the
    verifying endpoint -- CreateMultipartUpload (the upload ID from its XML), the six parts
    PUT to that upload, CompleteMultipartUpload listing every part's ETag in order
    (multipart_upload.cpp:48-61) -- and the object ETag the server computes from the MD5s of
    what it received equals the local multipart ETag from the part MD5s (and the compiled
    reference's md5 golden for this file).  Without MD5s the object ETag is reported only; a
    part the server answered with a wrong ETag makes Complete fail (InvalidPart)."""
    want = golden["md5"]["transfer_etag"]
    proc, url, stats = _start_mock()
    try:
        r, _ = _upload(args + ["--multipart", "--content-md5", "--repeat", "2"], url, tmp_path, golden)
        assert r.returncode == 0, r.stderr
        assert f"object etag {want} == the local multipart etag" in r.stderr, r.stderr
        assert "upload id upload-2" in r.stderr, r.stderr  # a fresh upload per pass
        r, _ = _upload(args + ["--multipart"], url, tmp_path, golden)
        assert r.returncode == 0 and f"object etag {want}" in r.stderr, r.stderr
        s = stats()
        assert s["creates"] == 3 and s["completes"] == 3 and s.get("bad_completes", 0) == 0, s
        assert s["parts"] == 18 and s["bad_hash"] == 0 and s["bad_signature"] == 0, s
        r, _ = _upload(args + ["--multipart", "--secret", "WRONG"], url, tmp_path, golden)
        assert r.returncode == 1 and "CreateMultipartUpload: HTTP status 403" in r.stderr, r.stderr
    finally:
        proc.kill()
        proc.wait()
    proc, url, stats = _start_mock("--wrong-etag-part", "4")
    try:
        r, _ = _upload(args + ["--multipart"], url, tmp_path, golden)
        assert r.returncode == 1 and "CompleteMultipartUpload: HTTP status 400" in r.stderr, r.stderr
        assert "InvalidPart" in r.stderr and stats()["bad_completes"] == 1
    finally:
        proc.kill()
        proc.wait()


def test_upload_multipart_flow_cpu(programs, tmp_path, golden):
    _multipart_round(["--cpu"], tmp_path, golden)


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["file", "memory"])
def test_upload_multipart_flow_gpu(programs, tmp_path, golden, source):
    """The same with SHA-256 and MD5 from the GPU's dual pass."""
    _multipart_round(["--source", source], tmp_path, golden)
