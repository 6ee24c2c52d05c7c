#!/usr/bin/env python3
"""BASELINE config 5 on loopback: apps/s3_upload_hash --send against tests/s3_mock_server.py
(MinIO and libcurl's headers are absent from this image).  For one file and part geometry it
times the whole upload pass -- hash every part, PUT every part with its digest signed into
x-amz-content-sha256, the server verifying each body's SHA-256 and signature -- with
  gpu            one batched GPU call (H2D included), then the job threads PUT,
  gpu_per_job    one GPU call per job thread, each job then PUTs its parts,
  cpu_shani      the lib/hash drop-in on the job threads (x86 SHA-NI),
  cpu_scalar     the same drop-in forced onto its scalar loop (S3H_CPU_SCALAR=1), the closest
                 in-product stand-in for lib/hash's own cost,
and, for scale, hash_only_gpu / hash_only_cpu_shani (the same calls without --send).  With
C5_MULTIPART=1 every upload runs the reference's whole UploadFile flow (--multipart:
CreateMultipartUpload, the parts, CompleteMultipartUpload; the object ETag is reported).
Usage: c5_loopback.py FILE JOBS PARTS_PER_JOB [REPEAT]; one JSON line per variant."""
import json
import os
import re
import subprocess
import sys
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "apps", "build", "s3-upload-hash")


def main():
    path, jobs, ppj = sys.argv[1], sys.argv[2], sys.argv[3]
    repeat = sys.argv[4] if len(sys.argv) > 4 else "3"
    err = open(os.environ.get("C5_SERVER_LOG", os.devnull), "w")
    srv = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "s3_mock_server.py"),
                            "--port", "0"], stdout=subprocess.PIPE, stderr=err, text=True)
    try:
        url = f"http://127.0.0.1:{int(srv.stdout.readline())}"
        send = ["--send"] + (["--multipart"] if os.environ.get("C5_MULTIPART") == "1" else [])
        variants = [("gpu", send, {}), ("gpu_per_job", send + ["--per-job"], {}),
                    ("cpu_shani", send + ["--cpu"], {}),
                    ("cpu_scalar", send + ["--cpu"], {"S3H_CPU_SCALAR": "1"}),
                    ("hash_only_gpu", [], {}), ("hash_only_cpu_shani", ["--cpu"], {})]
        for name, extra, env in variants:
            r = subprocess.run([APP, "-f", path, "-j", jobs, "-n", ppj, "--endpoint", url,
                                "--repeat", repeat, *extra], capture_output=True, text=True,
                               timeout=600, env={**os.environ, **env})
            rx = r"(\d+) parts, ([\d.]+) GiB in ([\d.]+) s = ([\d.]+) GiB/s"
            line = next((l for l in r.stderr.splitlines() if re.search(rx, l)), "")
            m = re.search(rx, line)
            me = re.search(r"object etag (\S+)", r.stderr)
            with urllib.request.urlopen(url + "/stats", timeout=10) as f:
                stats = json.loads(f.read())
            print(json.dumps({"variant": name, "rc": r.returncode, "jobs": int(jobs),
                              "parts": int(m.group(1)) if m else None,
                              "GiB": float(m.group(2)) if m else None,
                              "seconds": float(m.group(3)) if m else None,
                              "GiBps": float(m.group(4)) if m else None,
                              "object_etag": me.group(1) if me else None,
                              "server_totals": stats, "line": line}), flush=True)
            if r.returncode != 0:
                return 1
    finally:
        srv.kill()
        srv.wait()
    return 0


if __name__ == "__main__":
    sys.exit(main())
