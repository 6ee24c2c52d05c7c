"""Cut a `trace:tools/host_timeline.py` rocprofv3 trace into the host-path calls and say
where each call's time goes.

usage: python3 tools/host_timeline_summary.py PROF_DIR TIMELINE_LOG

The trace's timestamps and the script's time.monotonic_ns() are the same clock, so each
call's copies and kernels are the records inside [t0_ns, t1_ns].  Per call: the wall time,
the H2D copies' busy time and the idle gaps between them, start -> first copy, last copy ->
last kernel end, last kernel -> return, and the plain copy rate while copies ran."""
import csv
import json
import sys
from pathlib import Path


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(prof, log):
    prof = Path(prof)
    calls = json.loads(Path(log).read_text().strip().splitlines()[-1])["calls"]
    copies = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"])
              for r in rows(prof / "run_memory_copy_trace.csv")]
    kerns = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
             for r in rows(prof / "run_kernel_trace.csv")]
    out = []
    for c in calls:
        t0, t1 = c["t0_ns"], c["t1_ns"]
        h2d = sorted((a, b) for a, b, d in copies
                     if d.endswith("HOST_TO_DEVICE") and t0 <= a <= t1)
        d2h = sorted((a, b) for a, b, d in copies
                     if d.endswith("DEVICE_TO_HOST") and t0 <= a <= t1)
        ks = sorted((a, b, n.split("(")[0]) for a, b, n in kerns if t0 <= a <= t1)
        busy = sum(b - a for a, b in h2d)
        gaps = [h2d[i + 1][0] - h2d[i][1] for i in range(len(h2d) - 1)]
        last_k = max(b for a, b, _ in ks) if ks else t1
        last_any = max([last_k] + [b for _, b in d2h])
        ms = lambda x: round(x / 1e6, 3)  # noqa: E731
        out.append({
            "wall_ms": ms(t1 - t0), "h2d_copies": len(h2d), "kernels": len(ks),
            "kernel_names": sorted({n for _, _, n in ks}),
            "h2d_busy_ms": ms(busy), "h2d_gap_ms_total": ms(sum(gaps)),
            "h2d_gap_ms_max": ms(max(gaps) if gaps else 0),
            "start_to_first_copy_ms": ms(h2d[0][0] - t0) if h2d else None,
            "last_copy_to_last_kernel_end_ms": ms(last_k - h2d[-1][1]) if h2d else None,
            "last_gpu_op_to_return_ms": ms(t1 - last_any),
            "d2h_copies": len(d2h),
            "last_kernel_ms": ms(ks[-1][1] - ks[-1][0]) if ks else None,
        })
    print(json.dumps({"calls": out}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
