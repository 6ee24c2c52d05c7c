#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes for the SHA-256 kernels into profiles/<name>.json.

    python tools/pmc_summary.py --fetch DIR --write DIR [--sq DIR] --kernel-stats CSV \
        --bytes-per-launch B --bench-jsonl LINE --kernel-key skew --out profiles/r03_c2_skew_pmc.json

Provenance: the summary records the kernel's code hash and the library sha256 that the
profiled bench run loaded (its JSON line's `library` object, --bench-jsonl) and the git commit
it was summarised at; bench.py uses a profile's traffic only for a build whose kernel code
hash is the same (pmc_traffic).

HBM traffic follows MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE (KiB) come from
separate passes; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
read traffic = 2 * FETCH_SIZE * 1024 (the kernel's loads are 16 B/lane global_load_dwordx4).
"""
import argparse
import collections
import csv
import json
import os


def per_dispatch(d, kernel_substr):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if kernel_substr in r["Kernel_Name"]:
                agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def mean(agg, name):
    vals = [v[name] for v in agg.values() if name in v]
    return sum(vals) / len(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq")
    ap.add_argument("--kernel", default="sha256_")
    ap.add_argument("--kernel-stats")
    ap.add_argument("--bytes-per-launch", type=float, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--bench-jsonl", required=True,
                    help="the profiled bench.py run's output (its `library` object)")
    ap.add_argument("--kernel-key", required=True, help="tools/isa_counts.py ALL_KERNELS key")
    a = ap.parse_args()
    fetch = mean(per_dispatch(a.fetch, a.kernel), "FETCH_SIZE")
    write = mean(per_dispatch(a.write, a.kernel), "WRITE_SIZE")
    read_bytes = 2.0 * fetch * 1024.0
    write_bytes = write * 1024.0
    out = {"kernel_filter": a.kernel, "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "read_bytes_corrected": read_bytes, "write_bytes": write_bytes,
           "traffic_bytes_per_launch": read_bytes + write_bytes,
           "algorithmic_bytes_per_launch": a.bytes_per_launch,
           "traffic_over_algorithmic": (read_bytes + write_bytes) / a.bytes_per_launch,
           "correction": "FETCH_SIZE x2 (gfx950 reports half of a 16-B/lane streaming read)"}
    import subprocess
    line = json.loads(open(a.bench_jsonl).read().strip().splitlines()[-1])
    lib = line["library"]
    out["kernel_key"] = a.kernel_key
    out["kernel_code_hash"] = lib["kernel_code_hash"][a.kernel_key]
    out["library_sha256"] = lib["sha256"]
    out["library_path"] = lib["path"]
    head = subprocess.run(["git", "rev-parse", "HEAD"], capture_output=True, text=True).stdout.strip()
    dirty = subprocess.run(["git", "status", "--porcelain", "--untracked-files=no"],
                           capture_output=True, text=True).stdout.strip()
    out["git_head"] = head + ("+uncommitted" if dirty else "")
    if a.sq:
        sq = per_dispatch(a.sq, a.kernel)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_WAVE_CYCLES",
                  "SQ_BUSY_CYCLES"):
            out[c] = mean(sq, c)
    if a.kernel_stats:
        with open(a.kernel_stats) as f:
            for r in csv.DictReader(f):
                if a.kernel in r["Name"]:
                    out["kernel"] = r["Name"]
                    out["avg_duration_ns"] = float(r["AverageNs"])
                    out["calls"] = int(r["Calls"])
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
