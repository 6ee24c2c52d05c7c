#!/usr/bin/env python3
"""Loopback S3 UploadPart endpoint for BASELINE config 5 (test infrastructure, not product).

MinIO and the libcurl headers are absent from this image, so config 5 (apps/parallel_upload.cpp
end-to-end against MinIO on loopback) runs against this stand-in instead.  It accepts what
`apps/s3_upload_hash --send` PUTs -- S3Api::UploadPart / UploadFilePart requests
(`PUT /{bucket}/{key}?partNumber=N&uploadId=ID`, lib/src/api/multipart_upload.cpp:71-156) --
and checks each one the way an S3 server would:

* the body's SHA-256 (Python hashlib, independent of this repo's code) equals the
  `x-amz-content-sha256` header (400 XAmzContentSHA256Mismatch otherwise), and
* the SigV4 `Authorization` header verifies: the canonical request is rebuilt from the
  received method, path, query and the headers named in SignedHeaders, as
  lib/src/aws_sign.cpp:226-308 builds it (403 SignatureDoesNotMatch otherwise), and
* a `Content-MD5` header, when sent, is the base64 MD5 of the body (400 BadDigest otherwise).

A verified part gets 200 with `ETag: "<md5 of body>"` (what S3 returns for UploadPart).
With `--store` the parts are kept and a signed `GET /{bucket}/{key}` with `Range: bytes=a-b`
returns that range of the parts concatenated in part-number order (the ranged GETs of
lib/src/download.cpp:72-103); `--corrupt-get K` flips one byte of the K-th GET's body.
`--fail-every K` answers every K-th PUT with 503 SlowDown after reading it (to exercise the
uploader's retries, upload.cpp:55-87).  `--wrong-etag-part N` answers part N's PUTs with an
ETag that is not the body's MD5 (a server-side corruption the uploader's ETag check must
catch).  `GET /stats` returns JSON counts.  Run: `s3_mock_server.py --port 0 --port-file F` (prints
the bound port).

Multipart uploads (`s3_upload_hash --send --multipart`, the reference's UploadFile flow,
lib/src/upload.cpp:113-149): `POST ?uploads` (CreateMultipartUpload) answers an
`<UploadId>`; parts PUT to that upload are recorded with their MD5s; `POST ?uploadId=ID`
(CompleteMultipartUpload, multipart_upload.cpp:48-61 builds its XML) checks that every listed
part was received with the listed ETag, in ascending part order (400 InvalidPart /
InvalidPartOrder otherwise), and answers the object ETag S3 computes -- hex MD5 of the parts'
binary MD5s + "-" + part count -- quoted as `&quot;`.  Both POSTs are checked like PUTs
(body SHA-256 against x-amz-content-sha256, SigV4)."""
import argparse
import base64
import hashlib
import hmac
import json
import re
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

_UNRESERVED = "-_.~"


def _enc(s: str) -> str:  # url_utility.cpp:70-90: alnum and -_.~ kept, the rest %XX (upper)
    return "".join(c if (c.isascii() and c.isalnum()) or c in _UNRESERVED
                   else "".join(f"%{b:02X}" for b in c.encode()) for c in s)


def _hm(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def expected_signature(secret, method, path, query, headers, signed, payload, date, scope):
    """SigV4 as aws_sign.cpp:226-308 computes it (sorted query, 'name:value' header lines)."""
    params = urllib.parse.parse_qsl(query, keep_blank_values=True)
    cq = "&".join(f"{_enc(k)}={_enc(v)}" for k, v in sorted(params))
    block = "".join(f"{h}:{headers.get(h, '')}\n" for h in signed)
    creq = f"{method.upper()}\n{path}\n{cq}\n{block}\n{';'.join(signed)}\n{payload}"
    to_sign = ("AWS4-HMAC-SHA256\n" + date + "\n" + scope + "\n"
               + hashlib.sha256(creq.encode()).hexdigest())
    day, region, service, _ = scope.split("/")
    key = _hm(_hm(_hm(_hm(("AWS4" + secret).encode(), day), region), service), "aws4_request")
    return hmac.new(key, to_sign.encode(), hashlib.sha256).hexdigest()


class Server(ThreadingHTTPServer):
    request_queue_size = 256  # an uploader opens one connection per job at once
    daemon_threads = True


class Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    secret = "SECRET"
    stats = {"parts": 0, "bytes": 0, "bad_hash": 0, "bad_signature": 0, "short_body": 0,
             "injected_503": 0, "puts": 0, "md5_checked": 0, "bad_md5": 0}
    fail_every = 0
    store = False
    corrupt_get = 0
    wrong_etag_part = 0
    objects = {}  # "/bucket/key" -> {part number: bytes}
    uploads = {}  # upload id -> {"path": "/bucket/key", "parts": {part number: md5 hex}}
    gets = 0
    lock = threading.Lock()

    def log_message(self, *a):  # quiet
        pass

    def _reply(self, code, body=b"", etag=None):
        self.send_response(code)
        if etag:
            self.send_header("ETag", f'"{etag}"')
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _signature_ok(self, payload: str) -> bool:
        auth = self.headers.get("Authorization", "")
        try:
            fields = dict(kv.strip().split("=", 1) for kv in auth.split(" ", 1)[1].split(","))
            scope = fields["Credential"].split("/", 1)[1]
            signed = fields["SignedHeaders"].split(";")
            hdrs = {k.lower(): v for k, v in self.headers.items()}
            path, _, query = self.path.partition("?")
            want = expected_signature(self.secret, self.command, path, query, hdrs, signed,
                                      payload, hdrs.get("x-amz-date", ""), scope)
            return hmac.compare_digest(want, fields["Signature"])
        except (KeyError, IndexError, ValueError):
            return False

    def do_GET(self):
        if self.path == "/stats":
            with self.lock:
                body = json.dumps(self.stats).encode()
            return self._reply(200, body)
        if not self._signature_ok(self.headers.get("x-amz-content-sha256", "")):
            with self.lock:
                self.stats["bad_signature"] += 1
            return self._reply(403, b"SignatureDoesNotMatch")
        path = self.path.partition("?")[0]
        with self.lock:
            parts = self.objects.get(path)
            obj = b"".join(parts[k] for k in sorted(parts)) if parts else None
            Handler.gets += 1
            nth = Handler.gets
        if obj is None:
            return self._reply(404, b"NoSuchKey")
        rng = self.headers.get("Range", "")
        a, b = 0, len(obj) - 1
        if rng.startswith("bytes="):
            lo, _, hi = rng[6:].partition("-")
            a, b = int(lo), min(int(hi), len(obj) - 1) if hi else len(obj) - 1
        body = bytearray(obj[a:b + 1])
        if self.corrupt_get and nth == self.corrupt_get and body:
            body[len(body) // 2] ^= 0x01
        with self.lock:
            self.stats["gets"] = self.stats.get("gets", 0) + 1
        self._reply(206 if rng else 200, bytes(body))

    def do_PUT(self):
        n = int(self.headers.get("content-length", "0"))
        body = self.rfile.read(n)
        if len(body) != n:  # the client went away mid-body
            with self.lock:
                self.stats["short_body"] += 1
            self.close_connection = True
            return
        with self.lock:
            self.stats["puts"] += 1
            inject = self.fail_every > 0 and self.stats["puts"] % self.fail_every == 0
            if inject:
                self.stats["injected_503"] += 1
        if inject:
            return self._reply(503, b"SlowDown")
        claimed = self.headers.get("x-amz-content-sha256", "")
        digest = hashlib.sha256(body).hexdigest()
        if claimed != digest:
            with self.lock:
                self.stats["bad_hash"] += 1
            return self._reply(400, b"XAmzContentSHA256Mismatch")
        cmd5 = self.headers.get("Content-MD5")
        if cmd5 is not None:
            ok = cmd5 == base64.b64encode(hashlib.md5(body).digest()).decode()
            with self.lock:
                self.stats["md5_checked" if ok else "bad_md5"] += 1
            if not ok:
                return self._reply(400, b"BadDigest")
        if not self._signature_ok(claimed):
            with self.lock:
                self.stats["bad_signature"] += 1
            return self._reply(403, b"SignatureDoesNotMatch")
        path, _, query = self.path.partition("?")
        q = dict(urllib.parse.parse_qsl(query))
        pn = int(q.get("partNumber", "0"))
        etag = hashlib.md5(body).hexdigest()
        with self.lock:
            self.stats["parts"] += 1
            self.stats["bytes"] += n
            if self.store:
                self.objects.setdefault(path, {})[pn] = body
            up = self.uploads.get(q.get("uploadId", ""))
            if up is not None and up["path"] == path:
                up["parts"][pn] = etag
            if pn == self.wrong_etag_part:
                self.stats["wrong_etags"] = self.stats.get("wrong_etags", 0) + 1
                etag = hashlib.md5(body + b"x").hexdigest()
        self._reply(200, etag=etag)


    def _count(self, what):
        with self.lock:
            self.stats[what] = self.stats.get(what, 0) + 1

    def do_POST(self):
        n = int(self.headers.get("content-length", "0"))
        body = self.rfile.read(n)
        claimed = self.headers.get("x-amz-content-sha256", "")
        if len(body) != n or claimed != hashlib.sha256(body).hexdigest():
            self._count("bad_hash")
            return self._reply(400, b"XAmzContentSHA256Mismatch")
        if not self._signature_ok(claimed):
            self._count("bad_signature")
            return self._reply(403, b"SignatureDoesNotMatch")
        path, _, query = self.path.partition("?")
        q = dict(urllib.parse.parse_qsl(query, keep_blank_values=True))
        bucket, _, key = path.lstrip("/").partition("/")
        if "uploads" in q:  # CreateMultipartUpload
            with self.lock:
                uid = f"upload-{len(self.uploads) + 1}"
                self.uploads[uid] = {"path": path, "parts": {}}
                self.stats["creates"] = self.stats.get("creates", 0) + 1
            return self._reply(200, (
                '<?xml version="1.0" encoding="UTF-8"?>\n<InitiateMultipartUploadResult '
                'xmlns="http://s3.amazonaws.com/doc/2006-03-01/">'
                f"<Bucket>{bucket}</Bucket><Key>{key}</Key><UploadId>{uid}</UploadId>"
                "</InitiateMultipartUploadResult>").encode())
        uid = q.get("uploadId")
        with self.lock:
            up = self.uploads.get(uid)
        if up is None or up["path"] != path:
            self._count("bad_completes")
            return self._reply(404, b"NoSuchUpload")
        listed = re.findall(r"<Part>\s*<ETag>(.*?)</ETag>\s*<PartNumber>(\d+)</PartNumber>\s*</Part>",
                            body.decode(errors="replace"), re.S)
        numbers = [int(pn) for _, pn in listed]
        if not listed or numbers != sorted(set(numbers)):
            self._count("bad_completes")
            return self._reply(400, b"InvalidPartOrder")
        md5s = []
        for etag, pn in listed:
            etag = etag.strip().replace("&quot;", "").replace("&#34;", "").strip('"').lower()
            if up["parts"].get(int(pn)) != etag:
                self._count("bad_completes")
                return self._reply(400, b"InvalidPart")
            md5s.append(bytes.fromhex(etag))
        final = f"{hashlib.md5(b''.join(md5s)).hexdigest()}-{len(md5s)}"
        self._count("completes")
        self._reply(200, (
            '<?xml version="1.0" encoding="UTF-8"?>\n<CompleteMultipartUploadResult '
            'xmlns="http://s3.amazonaws.com/doc/2006-03-01/">'
            f"<Location>http://127.0.0.1{path}</Location><Bucket>{bucket}</Bucket><Key>{key}</Key>"
            f"<ETag>&quot;{final}&quot;</ETag></CompleteMultipartUploadResult>").encode())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--port-file", default="")
    ap.add_argument("--secret", default="SECRET")
    ap.add_argument("--fail-every", type=int, default=0)
    ap.add_argument("--store", action="store_true")
    ap.add_argument("--corrupt-get", type=int, default=0)
    ap.add_argument("--wrong-etag-part", type=int, default=0)
    a = ap.parse_args()
    Handler.wrong_etag_part = a.wrong_etag_part
    Handler.secret = a.secret
    Handler.fail_every = a.fail_every
    Handler.store = a.store
    Handler.corrupt_get = a.corrupt_get
    srv = Server(("127.0.0.1", a.port), Handler)
    port = srv.server_address[1]
    if a.port_file:
        with open(a.port_file, "w") as f:
            f.write(str(port))
    print(port, flush=True)
    srv.serve_forever()


if __name__ == "__main__":
    main()
