"""Pinned host -> HBM copy rate with one, two and four concurrent copy streams (each stream
copies its share of an 8 GiB pinned buffer in 256 MiB pieces), and the 2-D slice shape the
host path uses; best of 3 each, wall clock around the whole set.  Tells whether the host
path (one copy stream) leaves PCIe bandwidth unused.

usage: python3 tools/ubench_h2d.py [GIB]"""
import json
import sys
import time

import torch


def main():
    gib = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = gib << 30
    piece = 256 << 20
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    host.fill_(7)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    res = {}
    for ns in (1, 2, 4, 1):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        best = None
        for _ in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for k, o in enumerate(range(0, n, piece)):
                with torch.cuda.stream(streams[k % ns]):
                    dev[o:o + piece].copy_(host[o:o + piece], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        res.setdefault(f"{ns}_streams", []).append(round(gib / best, 3))
    print(json.dumps({"GiB": gib, "piece_MiB": piece >> 20, "GiBps_best_of_3": res}))


if __name__ == "__main__":
    main()
