#!/bin/bash
# Round-2 GPU pass AB: producers decode lanes without a part (partial last group) on the
# full-block path -- full GPU suite, then dual digest and SHA-256 at partial part counts:
# split grid (product for <= 1,820 parts) vs group kernel (experiment build), and the C2 line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_ab.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_ab.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_ab.log | head -20; exit 1; }
run() {  # tag, lib, mode, n
  S3H_LIBRARY=$2 timeout -k 10 300 python bench.py --mode $3 --steps 3 --warmup 1 --config c4 --parts-per-gpu $4 --no-cpu-baseline --no-host-resident > gpurun_out/bench_ab_$1.jsonl 2> gpurun_out/bench_ab_$1.err || { tail -20 gpurun_out/bench_ab_$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ab_$1.jsonl').read().strip().splitlines()[-1]); print('$1', d['value'], d.get('ms_per_batch', d.get('ms_per_step')), d.get('fixture_mismatches', d.get('parity')))"
}
for n in 1000 1800 2050; do
  run split_$n s3client_amd/lib/libs3hash.so dual $n
  run group_$n tools/exp/libs3hash_nosplit.so dual $n
  run sha_$n s3client_amd/lib/libs3hash.so device $n
done
run sha_4100 s3client_amd/lib/libs3hash.so device 4100
run dual_4100 s3client_amd/lib/libs3hash.so dual 4100
