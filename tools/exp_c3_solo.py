#!/usr/bin/env python3
"""Experiment (not the product): BASELINE config 3 (4,096 x U[5,64] MiB) on the two-group skew
kernel with the current library (S3H_LIBRARY selects a `make exp` variant), reporting the
kernel time and, from the clock probe, cycles per block of every group split into the groups
that ran alone on their workgroup (solo) and the paired ones.

    python tools/exp_c3_solo.py --steps 3 [--tag name]      -> one JSON line
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("S3H_LIBRARY", "product")))
    ap.add_argument("--parts", type=int, default=4096)
    args = ap.parse_args()
    import torch

    import s3client_amd as s3
    from bench import SEED, workload
    ids, lens, offs, name = workload("c3", 0, 1, args.parts, 0)
    dev = torch.device("cuda", 0)
    data = torch.empty(int(offs[-1] + lens[-1]) + 256, dtype=torch.uint8, device=dev)
    s3.generate_parts(data, offs, lens, ids, SEED)
    plan = s3.Plan(offs, lens, device=0)
    info = plan.info()
    dig = torch.zeros((len(lens), 8), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    plan.launch(data, dig, stream)
    torch.cuda.synchronize()
    ms = []
    for _ in range(args.steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        plan.launch(data, dig, stream)
        b.record(stream)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    clocks = torch.zeros(4 * 1024, dtype=torch.int64, device=dev)
    waves = plan.set_clock_probe(clocks)
    plan.launch(data, dig, stream)
    torch.cuda.synchronize()
    plan.set_clock_probe(None)
    c = clocks.view(-1, 4)[:waves].cpu().numpy().astype(np.float64)
    cyc, rt = c[:, 1] - c[:, 0], c[:, 3] - c[:, 2]
    srt = np.sort(lens.astype(np.int64))[::-1]
    gblocks = ((srt[::8] + 9 + 63) // 64)[:waves].astype(np.float64)
    cpb = cyc / gblocks
    # groups that ran alone: the grid has `grid` workgroups for `waves` groups
    solo = 2 * info["grid"] - waves
    ghz = float(np.median(cyc[rt > 0] / rt[rt > 0] * 0.1))
    # the groups that set the time: the slowest finishing ones (end time from the real-time
    # counter, relative to the earliest start)
    t_end = (c[:, 3] - c[:, 2].min()) / 1e5  # ms
    top = np.argsort(t_end)[::-1][:8]
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "sha256_golden.json")))
    fx = {e["p"]: e["digest"] for e in gold["c3_parts"]}
    gd = dig.cpu().numpy().view(np.uint32)
    bad = sum(s3.hash_to_text(gd[i]) != fx[int(p)] for i, p in enumerate(ids) if int(p) in fx)
    out = {"tag": args.tag, "kernel": info["kernel"], "grid": info["grid"], "groups": int(waves),
           "solo": int(solo), "kernel_ms": [round(x, 2) for x in ms],
           "GiBps": round(float(lens.sum()) / 2**30 / (min(ms) / 1e3), 2), "clock_GHz": round(ghz, 3),
           "cpb_solo_median": round(float(np.median(cpb[:solo])), 1) if solo else None,
           "cpb_paired_median": round(float(np.median(cpb[solo:])), 1),
           "cpb_paired_p90": round(float(np.percentile(cpb[solo:], 90)), 1),
           "cpb_group0": round(float(cpb[0]), 1),
           "last_groups": [[int(g), round(float(t_end[g]), 1), round(float(cpb[g]), 1)] for g in top],
           "fixtures": len([p for p in ids if int(p) in fx]), "mismatches": int(bad)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
