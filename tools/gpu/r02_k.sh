#!/bin/bash
# Round-2 GPU pass K: full regression (suite, smoke, default bench line) on the current tree.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_k.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_k.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_k.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_k.log 2>&1 || { tail -20 gpurun_out/smoke_k.log; exit 1; }
tail -1 gpurun_out/smoke_k.log
timeout -k 10 300 python bench.py > gpurun_out/bench_k.jsonl 2> gpurun_out/bench_k.err || { tail -20 gpurun_out/bench_k.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_k.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['issue']['frac'], d['host_resident']['value'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['parity'])"
