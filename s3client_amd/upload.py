"""Part geometry of the reference's parallel multipart upload, and per-part payload hashes.

``upload_parts_geometry`` restates how lib/src/upload.cpp slices an object into parts:
  * UploadFile / UploadData: perJobSize = ceil(size / jobs)       (upload.cpp:133, 168)
  * job i uploads parts [i*partsPerJob, (i+1)*partsPerJob)         (upload.cpp:136-140)
  * UploadParts: chunk = min(perJobSize, size - jobId*perJobSize);
    partSize = ceil(chunk / numParts); part k has min(partSize, chunk - k*partSize) bytes
    starting right after part k-1                                 (upload.cpp:98-107)
``payload_hashes`` produces the 64-char lowercase hex digests that the build passes as the
``payloadHash`` argument of S3Api::UploadFilePart (lib/include/s3-api.h:447-452) instead of
the reference's "UNSIGNED-PAYLOAD" (lib/src/aws_sign.cpp:236-237).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class UploadPart:
    job: int
    part_number: int   # firstPart + i, as passed to DoUploadPart (upload.cpp:104-106)
    offset: int
    size: int


def upload_parts_geometry(size: int, jobs: int, parts_per_job: int) -> list[UploadPart]:
    if size <= 0 or jobs <= 0 or parts_per_job <= 0:
        raise ValueError("size, jobs and parts_per_job must be positive")
    per_job = (size + jobs - 1) // jobs
    out: list[UploadPart] = []
    for job in range(jobs):
        offset = job * per_job
        if offset >= size:  # the reference would compute a negative chunk here; no parts
            continue
        chunk = min(per_job, size - offset)
        part_size = (chunk + parts_per_job - 1) // parts_per_job
        for k in range(parts_per_job):
            remaining = chunk - k * part_size
            if remaining <= 0:
                break
            s = min(part_size, remaining)
            out.append(UploadPart(job, job * parts_per_job + k, offset, s))
            offset += s
    return out


def payload_hashes(data, parts: list[UploadPart], ndevices: int = 0) -> list[str]:
    """GPU digests (hex) of each part of a host buffer, in ``parts`` order."""
    import numpy as np

    from .hashing import digests_to_text, sha256_batch_host
    buf = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data
    views = [buf[p.offset:p.offset + p.size] for p in parts]
    return digests_to_text(sha256_batch_host(views, ndevices=ndevices))
