"""Per-kernel table of one host-path call from a `trace:tools/host_timeline.py` run: start,
end, duration and the idle gap before each kernel, in ms from the call's start.

usage: python3 tools/host_timeline_kernels.py PROF_DIR TIMELINE_LOG [CALL_INDEX]"""
import csv
import json
import sys
from pathlib import Path


def main(prof, log, idx="1"):
    calls = json.loads(Path(log).read_text().strip().splitlines()[-1])["calls"]
    c = calls[int(idx)]
    t0, t1 = c["t0_ns"], c["t1_ns"]
    with open(Path(prof) / "run_kernel_trace.csv") as f:
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                    for r in csv.DictReader(f) if t0 <= int(r["Start_Timestamp"]) <= t1)
    print(f"# call {idx}: wall {c['ms']} ms ({c['GiBps']} GiB/s), {len(ks)} kernels")
    print("#  start_ms   end_ms    dur_ms  gap_ms  kernel")
    prev = None
    for a, b, n in ks:
        gap = 0.0 if prev is None else (a - prev) / 1e6
        print(f"{(a - t0) / 1e6:9.3f} {(b - t0) / 1e6:9.3f} {(b - a) / 1e6:8.3f} {gap:7.3f}  "
              f"{n.split('(')[0][:48]}")
        prev = b
    print(f"# return at {(t1 - t0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main(*sys.argv[1:4])
