#!/bin/bash
# Round-2 GPU pass U: shared-SIMD kernel with HW_ID-based consumer/producer pairing -- smoke,
# skews parity tests, C4 shard bench (skews, skewp) on one box.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_u.log 2>&1 || { tail -20 gpurun_out/smoke_u.log; exit 1; }
tail -1 gpurun_out/smoke_u.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "skews or c4_rank0 or shared_simd or dual_digest_group" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_u.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_u.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_u.log | head -20; exit 1; }
for k in auto skewp; do
  timeout -k 10 300 python bench.py --config c4 --kernel $k --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_u_$k.jsonl 2> gpurun_out/bench_c4_u_$k.err || { tail -20 gpurun_out/bench_c4_u_$k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_c4_u_$k.jsonl').read().strip().splitlines()[-1]); print('C4', d['config']['kernel'], d['value'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['clock_GHz'], d['parity'])"
done
