#!/bin/bash
# Round-2 GPU pass W: shared-SIMD producer writing W+K rows with ds_write_b128 (experiment,
# 16 LDS writes per block) vs the product's 64 ds_write_b32; C4 shard, interleaved.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # tag, lib
  S3H_LIBRARY=$2 timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_w_$1.jsonl 2> gpurun_out/bench_w_$1.err || { tail -20 gpurun_out/bench_w_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_w_$1.jsonl').read().strip().splitlines()[-1]); print('$1', d['config']['kernel'], d['value'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['clock_GHz'], d['parity'])"
}
run prod_a s3client_amd/lib/libs3hash.so
run rows_a tools/exp/libs3hash_rows.so
run prod_b s3client_amd/lib/libs3hash.so
run rows_b tools/exp/libs3hash_rows.so
