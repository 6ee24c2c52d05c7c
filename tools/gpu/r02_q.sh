#!/bin/bash
# Round-2 GPU pass Q: producer byte swap on the LDS pipe (product) vs VALU doublings
# (experiment) on the C4 shard; skews parity tests + smoke first.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_q.log 2>&1 || { tail -20 gpurun_out/smoke_q.log; exit 1; }
tail -1 gpurun_out/smoke_q.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "skews or c4_rank0 or dual_digest_group" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_q.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_q.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_q.log | head -20; exit 1; }
run() {  # tag, lib
  S3H_LIBRARY=$2 timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_$1.jsonl 2> gpurun_out/bench_c4_$1.err || { tail -20 gpurun_out/bench_c4_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_c4_$1.jsonl').read().strip().splitlines()[-1]); print('$1', d['config']['kernel'], d['value'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['cycles_per_instr'], d['issue']['clock_GHz'], d['parity'])"
}
run ldsbswap1 s3client_amd/lib/libs3hash.so
run valubswap1 tools/exp/libs3hash_valubswap.so
run ldsbswap2 s3client_amd/lib/libs3hash.so
run valubswap2 tools/exp/libs3hash_valubswap.so
