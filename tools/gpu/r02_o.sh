#!/bin/bash
# Round-2 GPU pass O: skews producer variants on the C4 shard (doubling byte swap = product,
# v_perm byte swap = experiment), 2 runs each, interleaved.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # tag, lib
  S3H_LIBRARY=$2 timeout -k 10 300 python bench.py --config c4 --kernel skews --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_$1.jsonl 2> gpurun_out/bench_c4_$1.err || { tail -20 gpurun_out/bench_c4_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_c4_$1.jsonl').read().strip().splitlines()[-1]); print('$1', d['value'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['cycles_per_instr'], d['issue']['clock_GHz'], d['parity'])"
}
run prod1 s3client_amd/lib/libs3hash.so
run perm1 tools/exp/libs3hash_permbswap.so
run prod2 s3client_amd/lib/libs3hash.so
run perm2 tools/exp/libs3hash_permbswap.so
