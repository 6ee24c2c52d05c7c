#!/bin/bash
# Round-2 GPU pass N: first run of the shared-SIMD producer kernel (skews): smoke, its parity
# tests, then C4 shard benches skews vs AUTO (skewp).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_n.log 2>&1 || { tail -20 gpurun_out/smoke_n.log; exit 1; }
tail -1 gpurun_out/smoke_n.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "skews or c4_rank0" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_n.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_n.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_n.log | head -20; exit 1; }
for k in skews auto; do
  timeout -k 10 300 python bench.py --config c4 --kernel $k --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_$k.jsonl 2> gpurun_out/bench_c4_$k.err || { tail -20 gpurun_out/bench_c4_$k.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_c4_$k.jsonl').read().strip().splitlines()[-1]); print('$k', d['value'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['cycles_per_instr'], d['parity'])"
done
