#!/bin/bash
# Round-2 GPU pass AA: dual digest split grid (product) vs group kernel (experiment build) over
# 512-1,800 parts of 8 MiB; SHA-256 alone for reference.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # tag, lib, mode, n
  S3H_LIBRARY=$2 timeout -k 10 300 python bench.py --mode $3 --steps 3 --warmup 1 --config c4 --parts-per-gpu $4 --no-cpu-baseline --no-host-resident > gpurun_out/bench_aa_$1.jsonl 2> gpurun_out/bench_aa_$1.err || { tail -20 gpurun_out/bench_aa_$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_aa_$1.jsonl').read().strip().splitlines()[-1]); print('$1', d['value'], d.get('ms_per_batch', d.get('ms_per_step')), d.get('fixture_mismatches', d.get('parity')))"
}
for n in 512 1024 1280 1536 1664 1800; do
  run split_$n s3client_amd/lib/libs3hash.so dual $n
  run group_$n tools/exp/libs3hash_nosplit.so dual $n
  run sha_$n s3client_amd/lib/libs3hash.so device $n
done
