"""s3h_sha256_file_parts at config 2's scale with different per-part pread sizes (the
`slice_bytes` argument), alternating in one process so every size sees the same page cache
and box: one 8 GiB file (random 64 MiB pattern repeated), 1,024 ranges of 8 MiB.  Prints one
JSON line per call and a summary line (median GiB/s per size); every call's digests must
equal the first call's.

usage: python3 tools/file_parts_ab.py [GIB] [SIZES_KIB] [ROUNDS] [SOURCE] [PART_MIB] [LIBRARY]  (defaults 8,
0,32,64,128,256, 3, file, 8; 0 = the library's own choice; SOURCE file = s3h_sha256_file_parts,
dual = s3h_sha256_md5_file_parts, memory = the file read into pageable RAM, then
s3h_sha256_batch_host over 1,024 views: host threads memcpy into the staging slot)"""
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 6:  # an experiment build (make exp) instead of the product library
    os.environ["S3H_LIBRARY"] = sys.argv[6]
import s3client_amd as s3  # noqa: E402


def main():
    gib = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    sizes = [int(x) << 10 for x in (sys.argv[2] if len(sys.argv) > 2 else "0,32,64,128,256").split(",")]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    source = sys.argv[4] if len(sys.argv) > 4 else "file"
    dual = source == "dual"
    path = os.path.join(tempfile.gettempdir(), f"s3h_ab_{gib}g.bin")
    block = np.random.default_rng(7).integers(0, 256, 64 << 20, dtype=np.uint8).tobytes()
    with open(path, "wb") as f:
        for _ in range(gib * 16):
            f.write(block)
    part = (int(sys.argv[5]) if len(sys.argv) > 5 else 8) << 20
    n = (gib << 30) // part
    offs = np.arange(n, dtype=np.uint64) * np.uint64(part)
    lens = np.full(n, part, dtype=np.uint64)
    fn = s3.sha256_md5_file_parts if dual else s3.sha256_file_parts
    if source == "memory":
        mem = np.fromfile(path, dtype=np.uint8)
        views = [mem[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]

        def fn(_path, _offs, _lens, slice_bytes=0):
            return s3.sha256_batch_host(views, slice_bytes=slice_bytes)
    try:
        ref = fn(path, offs, lens)  # warm: contexts, staging, code object
        ref = ref[0] if dual else ref
        for s in sizes:  # grow every size's ring once before timing
            fn(path, offs, lens, slice_bytes=s)
        res = {s: [] for s in sizes}
        for r in range(rounds):
            for s in sizes:
                t = time.perf_counter()
                out = fn(path, offs, lens, slice_bytes=s)
                dt = time.perf_counter() - t
                out = out[0] if dual else out
                ok = bool(np.array_equal(out, ref))
                res[s].append(gib / dt)
                print(json.dumps({"round": r, "slice_KiB": s >> 10, "GiBps": round(gib / dt, 3),
                                  "ms": round(1e3 * dt, 2), "digests_equal": ok}), flush=True)
                if not ok:
                    sys.exit(1)
        print(json.dumps({"summary": "median GiB/s per slice (KiB; 0 = library default)",
                          "source": source, "gib": gib, "parts": n,
                          "median": {s >> 10: round(float(np.median(v)), 3) for s, v in res.items()}}))
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
