#!/bin/bash
# Round-2 GPU pass Z: dual digest at 2,048 parts -- group kernel (product) vs two streams
# (experiment build), plus the dual tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "dual" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_z.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_z.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_z.log | head -20; exit 1; }
run() {  # tag, lib, args
  local tag=$1 lib=$2; shift 2
  S3H_LIBRARY=$lib timeout -k 10 400 python bench.py --mode dual --steps 3 --warmup 1 "$@" > gpurun_out/bench_z_$tag.jsonl 2> gpurun_out/bench_z_$tag.err || { tail -20 gpurun_out/bench_z_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_z_$tag.jsonl').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_batch'], d['fixture_mismatches'])"
}
run p2048_group s3client_amd/lib/libs3hash.so --config c4 --parts-per-gpu 2048
run p2048_2stream tools/exp/libs3hash_nogroupnc2.so --config c4 --parts-per-gpu 2048
run p1800_split s3client_amd/lib/libs3hash.so --config c4 --parts-per-gpu 1800
