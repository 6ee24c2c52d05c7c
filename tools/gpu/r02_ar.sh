#!/bin/bash
# Round-2 GPU pass AR: default bench line with the config-5 loopback and C3 / C4-shard sub-objects.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
( time timeout -k 10 400 python bench.py > gpurun_out/bench_ar.jsonl 2> gpurun_out/bench_ar.err ) 2> gpurun_out/bench_ar.time || { tail -20 gpurun_out/bench_ar.err; exit 1; }
cat gpurun_out/bench_ar.time
python3 -c "import json; d=json.loads(open('gpurun_out/bench_ar.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['host_resident']['value'], d['cpu_baseline']['value']); print(json.dumps(d['c5_loopback']['seconds'])); print(json.dumps(d['configs']))"
