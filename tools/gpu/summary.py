#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line (tools/gpu/run.sh): value, roofline fraction,
issue fraction, parity and the sub-measurements that are present."""
import json
import sys

line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [f"{line.get('metric', '')[:40]}: {line.get('value')} {line.get('unit', '')}"]
for k in ("roofline", "issue"):
    if isinstance(line.get(k), dict):
        out.append(f"{k}.frac {line[k].get('frac')}")
for k in ("parity", "status", "fixture_mismatches"):
    if k in line:
        out.append(f"{k} {line[k]}")
for k in ("host_resident", "cpu_baseline"):
    if isinstance(line.get(k), dict):
        out.append(f"{k} {line[k].get('value')}")
hr = line.get("host_resident") if isinstance(line.get("host_resident"), dict) else {}
for k in ("split", "stream"):
    if isinstance(hr.get(k), dict):
        out.append(f"host_resident.{k} {hr[k].get('GiBps')}")
if isinstance(line.get("configs"), dict):
    out.append("configs " + " ".join(f"{c}={v.get('GiBps')}" for c, v in line["configs"].items()))
if isinstance(line.get("c4"), dict):
    c4 = line["c4"]
    out.append(f"c4 agg {c4.get('aggregate_GiBps')} parity {c4.get('parity')}")
if "distinct_devices" in line:
    out.append(f"n_gpus {line.get('n_gpus')} distinct_devices {line['distinct_devices']}")
if line.get("errors"):
    out.append(f"ERRORS {line['errors']}")
print(" | ".join(out))
