#!/usr/bin/env python3
"""HBM traffic of a SHA-256 + MD5 dual grid from separate rocprofv3 --pmc passes
(tools/gpu/run.sh `pmc:FETCH_SIZE:...` and `pmc:WRITE_SIZE:...` of `bench.py --mode dual`).

    python tools/dual_pmc_summary.py --fetch DIR --write DIR --config c3 --kernel-key dual_group_mixed \
        --bench-jsonl LINE --out profiles/r06_c3_dual_mixed_pmc.json [--before profiles/OLD.json]

Read bytes = 2 x FETCH_SIZE KiB x 1024 (MI355X_MICROARCH.md gfx950 correction, 16-B/lane
loads); algorithmic bytes = every part read once + 32 B (SHA-256) + 16 B (MD5) written per
part.  The kernel's code hash and the library hash come from s3client_amd/kernel_isa_counts.json
(the build that ran: the GPU call pushed this tree's library)."""
import argparse
import collections
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SYMBOLS = {"dual_group_mixed": "sha256_md5_group_mixed_kernel",
           "dual_group": "sha256_md5_group_kernel<true>",
           "dual_group_skew": "sha256_md5_group_kernel<false>",
           "dual_split": "sha256_md5_dual_kernel"}


def per_dispatch(d, name, counter):
    agg = collections.defaultdict(float)
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if name in r["Kernel_Name"] and r["Counter_Name"] == counter:
                agg[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return [agg[k] for k in sorted(agg, key=int)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", required=True, choices=["c2", "c3", "c4"])
    ap.add_argument("--kernel-key", required=True, choices=sorted(SYMBOLS))
    ap.add_argument("--bench-jsonl", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--before", help="an earlier profile of the same grid, quoted beside")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    import bench
    _, lens, _, name = bench.workload(a.config, 0, 1, 0)
    algo = float(lens.sum()) + (32 + 16) * len(lens)
    sym = SYMBOLS[a.kernel_key]
    fetch = per_dispatch(a.fetch, sym, "FETCH_SIZE")
    write = per_dispatch(a.write, sym, "WRITE_SIZE")
    if not fetch or not write:
        sys.exit(f"no {sym} dispatches in the counter files")
    read_b = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    write_b = 1024.0 * sum(write) / len(write)
    isa = json.load(open(os.path.join(ROOT, "s3client_amd", "kernel_isa_counts.json")))
    line = json.loads(open(a.bench_jsonl).read().strip().splitlines()[-1])
    head = subprocess.run(["git", "rev-parse", "HEAD"], capture_output=True, text=True, cwd=ROOT).stdout.strip()
    out = {"what": f"{name}, SHA-256 + MD5 ({sym}): rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in "
                   f"separate passes of `bench.py --config {a.config} --mode dual`",
           "dispatches": len(fetch),
           "fetch_KiB_per_dispatch": [round(x, 1) for x in fetch],
           "write_KiB_per_dispatch": [round(x, 1) for x in write],
           "algorithmic_bytes_per_call": int(algo),
           "read_bytes": int(read_b), "write_bytes": int(write_b),
           "traffic_bytes_per_launch": int(read_b + write_b),
           "algorithmic_bytes_per_launch": int(algo),
           "traffic_over_algorithmic": round((read_b + write_b) / algo, 5),
           "correction": "FETCH_SIZE x2 (gfx950 reports half of a 16-B/lane read)",
           "kernel_key": a.kernel_key,
           "kernel_code_hash": isa["code_hash"].get(a.kernel_key),
           "library_sha256": isa.get("library_sha256"),
           "git_head": head + ("+uncommitted" if subprocess.run(
               ["git", "status", "--porcelain", "--untracked-files=no"], capture_output=True,
               text=True, cwd=ROOT).stdout.strip() else ""),
           "bench_line": {k: line.get(k) for k in ("metric", "value", "unit", "ms_per_batch")}}
    if a.before:
        b = json.load(open(a.before))
        out["before"] = {"file": a.before,
                         "read_over_algorithmic": b.get("read_over_algorithmic",
                                                        b.get("traffic_over_algorithmic"))}
    if a.note:
        out["note"] = a.note
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
