#!/bin/bash
# Round-2 GPU pass X: SHA-256 + MD5 for 2,049-4,096 parts through the group kernel (product)
# vs the two-stream path (experiment build = round-2 behaviour); dual tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "dual" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_x.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_x.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_x.log | head -20; exit 1; }
run() {  # tag, lib, args
  local tag=$1 lib=$2; shift 2
  S3H_LIBRARY=$lib timeout -k 10 400 python bench.py --mode dual --steps 2 --warmup 1 "$@" > gpurun_out/bench_x_$tag.jsonl 2> gpurun_out/bench_x_$tag.err || { tail -20 gpurun_out/bench_x_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_x_$tag.jsonl').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_batch'], d['fixture_mismatches'])"
}
run u4096_group s3client_amd/lib/libs3hash.so --config c4 --parts-per-gpu 4096
run u4096_2stream tools/exp/libs3hash_nogroupnc2.so --config c4 --parts-per-gpu 4096
run c3_group s3client_amd/lib/libs3hash.so --config c3
run c3_2stream tools/exp/libs3hash_nogroupnc2.so --config c3
