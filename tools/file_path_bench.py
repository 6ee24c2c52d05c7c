"""The upload app's file -> digest rate at config 2's scale: one 8 GiB file cut into 1,024
parts of 8 MiB (16 jobs x 64 parts, upload.cpp:89-110 geometry), hashed by
apps/build/s3-upload-hash from each source (`file` = pread into pinned staging, `mmap`,
`memory` = the whole file read into pageable RAM first), 3 passes each, with S3H_TRACE_HOST=1
so every call's setup / issue / drain split is logged.  The file is written once (random
64 MiB pattern repeated) and read from the page cache.  This process never touches the GPU;
the app is a child process.

usage: python3 tools/file_path_bench.py [GIB] [SOURCES]   (defaults: 8, file,mmap,memory)"""
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    gib = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    sources = (sys.argv[2] if len(sys.argv) > 2 else "file,mmap,memory").split(",")
    path = os.path.join(tempfile.gettempdir(), f"s3h_c2_{gib}g.bin")
    t = time.perf_counter()
    block = np.random.default_rng(7).integers(0, 256, 64 << 20, dtype=np.uint8).tobytes()
    with open(path, "wb") as f:
        for _ in range(gib * 16):
            f.write(block)
    print(f"wrote {gib} GiB in {time.perf_counter() - t:.1f} s", flush=True)
    app = os.path.join(ROOT, "apps", "build", "s3-upload-hash")
    env = dict(os.environ, S3H_TRACE_HOST="1")
    try:
        for src in sources:
            r = subprocess.run([app, "-f", path, "-j", "16", "-n", "64", "--source", src,
                                "--repeat", "3"], env=env, capture_output=True, text=True,
                               timeout=240)
            print(f"## source {src}: rc {r.returncode}", flush=True)
            print(r.stdout.strip())
            print(r.stderr.strip(), flush=True)
            if r.returncode:
                sys.exit(r.returncode)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
