#!/usr/bin/env python3
"""Per-launch kernel times of the default bench line's own rocprofv3 run (tools/gpu/run.sh
`stats`): `rocprofv3 --kernel-trace --stats -- python3 bench.py` writes the trace, and the
bench line it printed is the SAME process's.  Groups the trace by kernel and grid (the C2 skew
launches are the 128-workgroup sha256_skew_kernel<1> dispatches of ~121 ms; host-path slice
launches share the symbol but not the duration) and sets each group's mean beside the line's
own HIP-event figure, so the roofline's `achieved` can be checked against the profiler.

    python3 tools/same_run_summary.py STATS_DIR BENCH_JSONL OUT.json
"""
import csv
import json
import os
import subprocess
import sys


def launches(trace_csv, name_part, grid_x=None, min_ms=0.0):
    out = []
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            if name_part not in r["Kernel_Name"]:
                continue
            if grid_x is not None and int(r["Grid_Size_X"]) != grid_x:
                continue
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            if ms >= min_ms:
                out.append(ms)
    return out


def stats(ms):
    return {"launches": len(ms), "avg_ms": round(sum(ms) / len(ms), 3),
            "min_ms": round(min(ms), 3), "max_ms": round(max(ms), 3)} if ms else {"launches": 0}


def main():
    d, line_path, out_path = sys.argv[1:4]
    trace = os.path.join(d, "run_kernel_trace.csv")
    line = json.loads(open(line_path).read().strip().splitlines()[-1])
    roof = line["roofline"]
    # C2: 1,024 parts on the skew kernel = 128 workgroups of 128 threads (consumer + producer)
    c2 = launches(trace, "sha256_skew_kernel<1, false>", grid_x=128 * 128, min_ms=50.0)
    s = stats(c2)
    res = {"what": "rocprofv3 --kernel-trace --stats of `python3 bench.py` (the default N=1 line); "
                   "per-launch durations from its kernel trace, the line from the same process",
           "commit": subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                    text=True).stdout.strip(),
           "library_sha256": line["library"]["sha256"],
           "kernel_code_hash": line["library"]["kernel_code_hash"],
           "c2_skew": {**s, "bench_hip_event_kernel_ms": roof["kernel_ms"],
                       "achieved_GBps_from_trace": round(roof["bytes_per_launch"] / (s["avg_ms"] / 1e3) / 1e9, 2),
                       "roofline_frac_from_trace": round(roof["bytes_per_launch"] / (s["avg_ms"] / 1e3) / 1e9 / roof["peak"], 5),
                       "line_achieved_GBps": roof["achieved"], "line_frac": roof["frac"],
                       "line_traffic": roof["traffic"], "line_traffic_source": roof.get("traffic_source")}}
    cfg = line.get("configs", {})
    if "c3" in cfg:
        res["c3_skew_pairs"] = {**stats(launches(trace, "sha256_skew_pairs_kernel", min_ms=100.0)),
                                "bench_kernel_ms": cfg["c3"].get("kernel_ms")}
        res["c3_sha256_md5_mixed"] = {**stats(launches(trace, "sha256_md5_group_mixed_kernel", min_ms=100.0)),
                                      "bench_ms_per_call": cfg["c3"].get("sha256_md5", {}).get("ms_per_call")}
    if "c4" in cfg:
        ks = cfg["c4"].get("kernels", {})
        res["c4_skews"] = {**stats(launches(trace, "sha256_skew_shared_kernel", min_ms=50.0)),
                           "bench_kernel_ms": ks.get("skews", {}).get("kernel_ms")}
        res["c4_skewp"] = {**stats(launches(trace, "sha256_skew_kernel<1, true>", min_ms=50.0)),
                           "bench_kernel_ms": ks.get("skewp", {}).get("kernel_ms")}
    if "f_rows" in line:
        res["c2_md5_pc"] = {**stats(launches(trace, "md5_pc_kernel<4>", min_ms=20.0)),
                            "bench_kernel_ms": line["f_rows"].get("md5", {}).get("kernel_ms")}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
