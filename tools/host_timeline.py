"""Timeline of the host-resident path on the C2 batch, for a rocprofv3 kernel + memory-copy
trace: `rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run --
python3 tools/host_timeline.py`.  Prints one JSON line with each call's wall-clock bounds
(perf_counter and the trace's clock) so tools/host_timeline_summary.py can cut the trace
into calls and measure, per call: start -> first copy, gaps between copies, last copy ->
last kernel, last kernel -> return."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import s3client_amd as s3  # noqa: E402

MIB = 1 << 20


def main():
    n, L = int(os.environ.get("PARTS", "1024")), 8 * MIB
    dev = torch.device("cuda", 0)
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    lens = np.full(n, L, dtype=np.uint64)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    s3.generate_parts(buf, offs, lens, np.arange(n), 20241008)
    host = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    host.copy_(buf)
    want = s3.sha256_batch_device(buf, offs, lens).cpu().numpy().view(np.uint32)
    del buf
    torch.cuda.empty_cache()
    h = host.numpy()
    views = [h[int(o):int(o) + L] for o in offs]
    s3.sha256_batch_host(views, ndevices=1)
    calls = []
    for _ in range(int(os.environ.get("REPS", "3"))):
        time.sleep(0.05)  # a quiet gap in the trace between calls
        t0n, t0 = time.monotonic_ns(), time.perf_counter()
        out = s3.sha256_batch_host(views, ndevices=1)
        t1, t1n = time.perf_counter(), time.monotonic_ns()
        calls.append({"t0_ns": t0n, "t1_ns": t1n, "ms": round(1e3 * (t1 - t0), 3),
                      "GiBps": round(n * L / 2**30 / (t1 - t0), 3),
                      "ok": bool(np.array_equal(out, want))})
    print(json.dumps({"parts": n, "part_bytes": L, "calls": calls}))


if __name__ == "__main__":
    main()
